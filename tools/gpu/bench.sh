# the default bench line (or with extra bench.py args), detail object in its own file
#   bash tools/gpu/bench.sh <tag> [bench args]  ->  $O/bench.json (both stdout lines), $O/bench_detail.json
source "$(dirname "$0")/common.sh"
timeout -k 10 900 python -u bench.py --detail-out $O/bench_detail.json "$@" > $O/bench.json 2> $O/bench.err
echo bench done
