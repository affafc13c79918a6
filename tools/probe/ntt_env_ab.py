#!/usr/bin/env python3
"""NTT variant timing by environment knob (e.g. ZKP_NTT_RTAB=0 vs 1): for each configuration
("K=V K2=V2 ..."), the 2^23 and 2^20 coset-extension times of zkp_bench_ntt in a child process,
alternating the configurations for R rounds.  usage: ntt_env_ab.py R cfg1 [cfg2 ...]"""
import json, os, subprocess, sys

CHILD = r'''
import json, sys
sys.path.insert(0, "zk-p2p-onramp_amd")
import zkp_amd
r = {"cfg": sys.argv[1]}
for k in (23, 20):
    r["ms_%d" % k] = round(min(zkp_amd.bench_ntt(k, warmup=3, iters=20) for _ in range(3)), 4)
print(json.dumps(r))
'''


def main():
    rounds, cfgs = int(sys.argv[1]), sys.argv[2:]
    for _ in range(rounds):
        for cfg in cfgs:
            env = dict(os.environ)
            env.update(kv.split("=", 1) for kv in cfg.split())
            out = subprocess.run([sys.executable, "-c", CHILD, cfg], env=env, capture_output=True, text=True,
                                 timeout=300)
            line = [l for l in out.stdout.splitlines() if l.startswith("{")]
            print(line[0] if line else json.dumps({"cfg": cfg, "rc": out.returncode, "err": out.stderr[-400:]}),
                  flush=True)


if __name__ == "__main__":
    main()
