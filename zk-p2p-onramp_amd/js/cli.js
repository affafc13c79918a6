#!/usr/bin/env node
'use strict';
/*
 * CLI with snarkjs' argv shape (reference dizkus-scripts/5_gen_proof.sh:8, rapidsnark's
 * twin at 6_gen_proof_rapidsnark.sh:26):
 *   node cli.js groth16 prove <circuit.zkey> <witness.wtns> <proof.json> <public.json>
 * Output files are JSON.stringify(x, null, 1), byte-identical in layout to snarkjs.
 * and snarkjs' calldata export (reference circuit/scripts/generate_calldata.sh:3):
 *   node cli.js zkey export soliditycalldata <public.json> <proof.json>
 * and snarkjs' setup step (reference dizkus-scripts/3_gen_chunk_zkey.sh:18, `groth16 setup`):
 *   node cli.js groth16 setup|zkey new <circuit.r1cs> <pot.ptau> <circuit_0000.zkey> [-e=...]
 * a contribution and the final beacon (3_gen_chunk_zkey.sh:27,36; the record is appended to section 10):
 *   node cli.js zkey contribute <in.zkey> <out.zkey> -e=<entropy> [-n=name]
 *   node cli.js zkey beacon <in.zkey> <out.zkey> <beaconHashHex> <numIterationsExp> [-n=name]
 */
const fs = require('fs');
const { groth16, exportSolidityCallData, newZKey, beacon, contribute, release } = require('./groth16');

const USAGE = 'usage: cli.js groth16 prove <circuit.zkey> <witness.wtns> <proof.json> <public.json>\n' +
              '       cli.js zkey export soliditycalldata <public.json> <proof.json>\n' +
              '       cli.js groth16 setup|zkey new <circuit.r1cs> <pot.ptau> <circuit_0000.zkey>\n' +
              '       cli.js zkey contribute <in.zkey> <out.zkey> -e=<entropy> [-n=name]\n' +
              '       cli.js zkey beacon <in.zkey> <out.zkey> <beaconHashHex> <numIterationsExp> [-n=name]\n';

async function main(argv) {
  if (argv.length === 5 && argv[0] === 'zkey' && argv[1] === 'export' && argv[2] === 'soliditycalldata') {
    const pub = JSON.parse(fs.readFileSync(argv[3], 'utf-8'));
    const proof = JSON.parse(fs.readFileSync(argv[4], 'utf-8'));
    process.stdout.write(await exportSolidityCallData(proof, pub) + '\n');
    return 0;
  }
  const setupArgs = argv.filter((a) => !a.startsWith('-e='));  // entropy: unused by `groth16 setup`
  if (setupArgs.length === 5 && ((argv[0] === 'zkey' && argv[1] === 'new') || (argv[0] === 'groth16' && argv[1] === 'setup'))) {
    await newZKey(setupArgs[2], setupArgs[3], setupArgs[4]);
    return 0;
  }
  const named = argv.filter((a) => !/^(-n|--name)=/.test(a) && a !== '-v' && a !== '--verbose');
  if (argv[0] === 'zkey' && argv[1] === 'contribute') {
    const pos = argv.filter((a) => !a.startsWith('-'));
    const ent = argv.find((a) => /^(-e|--entropy)=/.test(a));
    const nameArg = argv.find((a) => /^(-n|--name)=/.test(a));
    if (pos.length === 4 && ent) {
      await contribute(pos[2], pos[3], nameArg ? nameArg.replace(/^[^=]*=/, '') : '', ent.replace(/^[^=]*=/, ''));
      return 0;
    }
  }
  if (named.length === 6 && argv[0] === 'zkey' && argv[1] === 'beacon') {
    const nameArg = argv.find((a) => /^(-n|--name)=/.test(a));
    await beacon(named[2], named[3], nameArg ? nameArg.replace(/^[^=]*=/, '') : '', named[4], named[5]);
    return 0;
  }
  if (argv.length !== 6 || argv[0] !== 'groth16' || argv[1] !== 'prove') {
    process.stderr.write(USAGE);
    return 1;
  }
  const [, , zkey, wtns, proofOut, publicOut] = argv;
  const { proof, publicSignals } = await groth16.prove(zkey, wtns);
  fs.writeFileSync(proofOut, JSON.stringify(proof, null, 1), 'utf-8');
  fs.writeFileSync(publicOut, JSON.stringify(publicSignals, null, 1), 'utf-8');
  release();
  return 0;
}

main(process.argv.slice(2)).then((c) => process.exit(c), (e) => {
  process.stderr.write(String(e && e.stack || e) + '\n');
  process.exit(1);
});
