# Round-2 check: full GPU suite (incl. the full-size parity tests), then the default bench.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python3 -c "import os;print('nproc',len(os.sched_getaffinity(0)),'cpu_count',os.cpu_count());print(open('/sys/fs/cgroup/cpu.max').read() if os.path.exists('/sys/fs/cgroup/cpu.max') else 'no cpu.max')" > gpurun_out/host.txt 2>&1 || true
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gt.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1
