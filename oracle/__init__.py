"""CPU oracle for the Groth16 `prove` hot path — TEST INFRASTRUCTURE ONLY.

Nothing under ``oracle/`` is part of the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import,
link or execute it, and only as the checker (never as the thing measured or
shipped).  The product path (``zk-p2p-onramp_amd/``) never imports it and fails
loudly when its HIP library is missing.

What it restates (SURVEY.md §8a rows A1–A11).  The reference itself holds no
prover code: the path lives in ``snarkjs@0.4.22`` → ``ffjavascript@0.2.55`` →
``wasmcurves@0.1.0`` (pins: reference ``package-lock.json:3884-3896``,
``:2060-2071``, ``:2081-2085``), none of which is present offline.  The oracle
therefore restates the published algorithm of those packages:

* ``bn254``    — Fq/Fr/Fq2/Fq6/Fq12 arithmetic, G1/G2, optimal-ate pairing
                 (ffjavascript tower: Fq6 = Fq2[v]/(v^3-(9+u)), Fq12 = Fq6[w]/(w^2-v)).
* ``ntt``      — ffjavascript root-of-unity convention (Fr.w[k]) and fft/ifft.
* ``binfile``  — snarkjs ``.zkey`` (v1, groth16) / ``.wtns`` (v2) sectioned files.
* ``circuit``  — seeded synthetic satisfiable R1CS ("Venmo-shaped" at any size).
* ``setup``    — INSECURE known-tau Groth16 setup producing snarkjs-layout zkeys.
* ``groth16``  — prover (A1–A10 with injectable r, s) and the ``Verifier.sol:340-358``
                 verification equation; snarkjs JSON formatting.

Pinning (see DESIGN.md "Oracle"): the pairing reproduces ``vk_alphabeta_12``
of ``app/src/helpers/vkey.ts:52-82`` from its own ``vk_alpha_1``/``vk_beta_2``;
the curve constants match ``contracts/Verifier.sol:52,341``; every vkey / IC
point of ``vkey.ts`` and ``Verifier.sol`` is on-curve; every oracle proof
verifies under the restated ``Verifier.sol`` equation.  No reference test pins a
prover output (the only proof fixture, ``test/ramp.test.js:193-196``, does not
verify — SURVEY.md §0.3), so the proof bytes themselves are pinned by the math
(A, B, C are a deterministic function of zkey, witness, r, s) plus verification.
"""
