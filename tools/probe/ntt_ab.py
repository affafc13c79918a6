#!/usr/bin/env python3
"""NTT variant timing: for each library given (ZKP_LIB_PATH per child process), the 2^23 and
2^20 coset-extension times of zkp_bench_ntt, alternating the libraries for R rounds.
usage: ntt_ab.py R lib1 [lib2 ...]"""
import json, os, subprocess, sys

CHILD = r'''
import json, sys
sys.path.insert(0, "zk-p2p-onramp_amd")
import zkp_amd
r = {"lib": sys.argv[1]}
for k in (23, 20):
    r["ms_%d" % k] = min(zkp_amd.bench_ntt(k, warmup=3, iters=20) for _ in range(3))
print(json.dumps(r))
'''

def main():
    rounds, libs = int(sys.argv[1]), sys.argv[2:]
    for _ in range(rounds):
        for lib in libs:
            env = dict(os.environ, ZKP_LIB_PATH=os.path.abspath(lib))
            out = subprocess.run([sys.executable, "-c", CHILD, lib], env=env, capture_output=True, text=True,
                                 timeout=300)
            line = [l for l in out.stdout.splitlines() if l.startswith("{")]
            print(line[0] if line else json.dumps({"lib": lib, "rc": out.returncode, "err": out.stderr[-400:]}),
                  flush=True)

if __name__ == "__main__":
    main()
