#!/usr/bin/env python3
"""One short NTT run for rocprofv3 passes: zkp_bench_ntt(log_n), 3 timed runs (or argv[2]).
usage: ntt_run.py [log_n=23] [iters=3]"""
import sys
sys.path.insert(0, "zk-p2p-onramp_amd")
import zkp_amd
k = int(sys.argv[1]) if len(sys.argv) > 1 else 23
print(zkp_amd.bench_ntt(k, warmup=1, iters=int(sys.argv[2]) if len(sys.argv) > 2 else 3))
