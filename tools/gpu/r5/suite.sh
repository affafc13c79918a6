# round 5: the whole GPU suite, smoke() and the default bench line on the round-5 library
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gt_suite.log 2>&1
echo suite done
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo smoke done
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
echo bench done
