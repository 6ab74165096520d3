#!/bin/bash
# GPU-box test run: the given pytest selection first, then the whole gpu suite.
#   gpurun -- bash scripts/job_tests.sh TAG [pytest args...]
TAG=${1:-t}
shift
SEL=${*:-tests}
exec bash scripts/gpu_job.sh "$TAG" \
  "sel:300:python -u -m pytest $SEL -m gpu -x -v --timeout 120 --timeout-method thread" \
  "all:420:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread"
