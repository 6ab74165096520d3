#!/bin/bash
# Test infrastructure: compile the reference's C++ growth simulator
# (/root/reference/src/mycelium_sim_2D.cpp, one self-contained file, standard
# library only) where it lies, into oracle/_ref/.  It is the checker of the
# native network producer (host/mfea_grow.cpp): the producer run
# with the same seed and parameters must write byte-identical nodes.csv /
# elements.csv.  Never shipped, never on the product path.  Needs
# /root/reference (this container only); the GPU box never runs it.
set -eu
HERE=$(cd "$(dirname "$0")" && pwd)
SRC=${REF_ROOT:-/root/reference}/src/mycelium_sim_2D.cpp
[ -f "$SRC" ] || { echo "reference source $SRC absent; oracle/_ref not built" >&2; exit 0; }
mkdir -p "$HERE/_ref"
# the reference's own compile line (mycelium_sim_2D.cpp:4)
g++ -O2 -std=c++17 "$SRC" -o "$HERE/_ref/mycelium_sim_2D"
echo "built $HERE/_ref/mycelium_sim_2D"
