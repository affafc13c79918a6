#!/usr/bin/env node
'use strict';
/*
 * CLI with snarkjs' argv shape (reference dizkus-scripts/5_gen_proof.sh:8, rapidsnark's
 * twin at 6_gen_proof_rapidsnark.sh:26):
 *   node cli.js groth16 prove <circuit.zkey> <witness.wtns> <proof.json> <public.json>
 * Output files are JSON.stringify(x, null, 1), byte-identical in layout to snarkjs.
 * and snarkjs' calldata export (reference circuit/scripts/generate_calldata.sh:3):
 *   node cli.js zkey export soliditycalldata <public.json> <proof.json>
 */
const fs = require('fs');
const { groth16, exportSolidityCallData, release } = require('./groth16');

const USAGE = 'usage: cli.js groth16 prove <circuit.zkey> <witness.wtns> <proof.json> <public.json>\n' +
              '       cli.js zkey export soliditycalldata <public.json> <proof.json>\n';

async function main(argv) {
  if (argv.length === 5 && argv[0] === 'zkey' && argv[1] === 'export' && argv[2] === 'soliditycalldata') {
    const pub = JSON.parse(fs.readFileSync(argv[3], 'utf-8'));
    const proof = JSON.parse(fs.readFileSync(argv[4], 'utf-8'));
    process.stdout.write(await exportSolidityCallData(proof, pub) + '\n');
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
