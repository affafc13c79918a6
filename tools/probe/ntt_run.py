#!/usr/bin/env python3
"""One short NTT run for rocprofv3 counter passes: zkp_bench_ntt(log_n) a few times."""
import sys
sys.path.insert(0, "zk-p2p-onramp_amd")
import zkp_amd
k = int(sys.argv[1]) if len(sys.argv) > 1 else 23
print(zkp_amd.bench_ntt(k, warmup=1, iters=3))
