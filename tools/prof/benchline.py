"""Read a bench.py output file: the detailed object (the {"bench_detail": ...} line that round 6's bench prints
before its compact contract line), or, for older files whose last line carried everything, that line."""
import json


def detail(path):
    lines = [l for l in open(path).read().strip().splitlines() if l.startswith("{")]
    for l in reversed(lines):
        d = json.loads(l)
        if "bench_detail" in d:
            return d["bench_detail"]
    return json.loads(lines[-1])
