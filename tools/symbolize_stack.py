"""Map the bare addresses of a signal-handler stack trace (glog style, as the
rocprofv3 tool prints it) to library + offset, using the memory map of a
clean run of the same command (tools/maps_bench.py writes one).

Libraries mapped at process start (libc, the preloaded tracer libraries, the
HSA runtime) keep their relative placement from run to run; only the ASLR
base moves.  The anchor is the signal trampoline __restore_rt in libc (the
frame right below the handler), found by its `mov $0xf,%rax; syscall`.

    python3 tools/symbolize_stack.py gpurun_out/f3_prof.log gpurun_out/maps_<pid>.txt
"""
import re
import subprocess
import sys


def restore_rt_offset(libc):
    out = subprocess.run(["objdump", "-d", libc], capture_output=True, text=True).stdout
    m = re.search(r"^\s*([0-9a-f]+):\s+48 c7 c0 0f 00 00 00\s+mov\s+\$0xf,%rax", out, re.M)
    return int(m.group(1), 16)


def load_maps(path):
    segs = []
    for line in open(path):
        f = line.split()
        if len(f) >= 6 and f[5].startswith("/"):
            lo, hi = (int(x, 16) for x in f[0].split("-"))
            segs.append((lo, hi, int(f[2], 16), f[5], f[1]))
    return segs


def main(log, maps):
    frames = [int(x, 16) for x in re.findall(r"@\s+0x([0-9a-f]+)", open(log).read())]
    pc = re.search(r"PC: @\s+0x([0-9a-f]+)", open(log).read())
    segs = load_maps(maps)
    libc = next(s for s in segs if "/libc.so" in s[3])
    base_now = min(s[0] for s in segs if s[3] == libc[3])
    restore = restore_rt_offset(libc[3])
    tramp = next(a for a in frames if (a - restore) & 0xfff == 0)  # page-aligned libc base
    delta = (tramp - restore) - base_now
    bases = {}
    for lo, hi, off, path, perm in segs:
        bases.setdefault(path, lo - off)
    print(f"libc base in the crashed run {tramp - restore:#x}, here {base_now:#x}")
    for a in ([int(pc.group(1), 16)] if pc else []) + frames:
        now = a - delta
        hit = next(((p, now - bases[p], perm) for lo, hi, off, p, perm in segs if lo <= now < hi), None)
        print(f"{a:#x} -> " + (f"{hit[0].rsplit('/', 1)[-1]} +{hit[1]:#x} ({hit[2]})" if hit else "?"))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
