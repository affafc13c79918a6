# the whole GPU test suite and __graft_entry__.smoke() on the in-tree library
#   bash tools/gpu/suite.sh <tag> [extra pytest args]  ->  $O/gpu_tests.txt, $O/smoke.txt
source "$(dirname "$0")/common.sh"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > $O/gpu_tests.txt 2>&1
echo suite done
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
echo smoke done
