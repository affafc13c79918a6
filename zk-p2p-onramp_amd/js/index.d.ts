// Type declarations for the zkp_amd Node host layer (no tsc in the build image; this
// documents the contract a TypeScript caller such as app/src/helpers/zkp.ts sees).
export type Input = string | { type: 'mem'; data: Uint8Array };
export interface Proof {
  pi_a: [string, string, '1'];
  pi_b: [[string, string], [string, string], ['1', '0']];
  pi_c: [string, string, '1'];
  protocol: 'groth16';
  curve: 'bn128';
}
export interface ProveOptions { devices?: number[]; r?: bigint | string; s?: bigint | string }
export interface Logger { debug?(msg: string): void; info?(msg: string): void }
export interface BatchOptions { devices?: number[]; rs?: (bigint | string)[]; ss?: (bigint | string)[] }
export declare const groth16: {
  prove(zkeyFileName: Input, witnessFileName: Input, logger?: Logger, opts?: ProveOptions):
    Promise<{ proof: Proof; publicSignals: string[] }>;
  // one entry per witness: the proof, or an Error (code = zkp_status) for a witness that failed
  proveBatch(zkeyFileName: Input, witnesses: Input[], logger?: Logger, opts?: BatchOptions):
    Promise<({ proof: Proof; publicSignals: string[] } | Error)[]>;
};
export declare function proveBatch(zkey: Input, witnesses: Input[], logger?: Logger, opts?: BatchOptions):
  Promise<({ proof: Proof; publicSignals: string[] } | Error)[]>;
export declare function prove(zkey: Input, wtns: Input, logger?: Logger, opts?: ProveOptions):
  Promise<{ proof: Proof; publicSignals: string[] }>;
export declare const zKey: {
  exportSolidityCallData(proof: Proof, publicSignals: string[]): Promise<string>;
  /** `snarkjs zkey new` on the GPU; writes zkeyName when given, returns the key bytes */
  newZKey(r1csName: Input, ptauName: Input, zkeyName?: string | { type: "mem"; data?: Uint8Array }, logger?: Logger,
          device?: number): Promise<Buffer>;
  /** `snarkjs zkey beacon`'s group arithmetic on the GPU (no transcript record appended) */
  beacon(zkeyNameOld: Input, zkeyNameNew: string | { type: "mem"; data?: Uint8Array } | undefined, name: string,
         beaconHashStr: string, numIterationsExp: number, logger?: Logger, device?: number): Promise<Buffer>;
};
export declare function exportSolidityCallData(proof: Proof, publicSignals: string[]): Promise<string>;
export declare function onRampArgs(proof: Proof, publicSignals: string[]):
  [[string, string], [[string, string], [string, string]], [string, string], string[]];
export declare function release(): void;
export declare function version(): string;
