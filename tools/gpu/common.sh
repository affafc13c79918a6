# sourced by every driver: run from the repo root on the GPU box, outputs under gpurun_out/<tag>/
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:?usage: bash tools/gpu/<driver>.sh <tag> [args]}
shift
O=gpurun_out/$TAG
mkdir -p "$O"
# the short bench command the profile passes run (one proof per step, no batch / kernels / CPU lines)
SHORT="python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line --sustain-s 0"
