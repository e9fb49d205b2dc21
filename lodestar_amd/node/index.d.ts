/**
 * Type declarations of @lodestar/blsgpu.  BlsGpuVerifier implements the shape of the beacon
 * node's IBlsVerifier (packages/beacon-node/src/chain/bls/interface.ts:20-46) over the
 * ISignatureSet union (packages/state-transition/src/util/signatureSets.ts:5-22), with one
 * widening: a pubkey may be a validator index into the device cache (or a PublicKey tagged
 * with .index by the pubkey-added hook) as well as a key object or 96-byte record.
 */

/** interface.ts:3-18 */
export interface VerifySignatureOpts {
  batchable?: boolean;
  verifyOnMainThread?: boolean;
}

/** interface.ts:20-46 */
export interface IBlsVerifier {
  verifySignatureSets(sets: ISignatureSet[], opts?: VerifySignatureOpts): Promise<boolean>;
  close(): Promise<void>;
}

export declare const SignatureSetType: {readonly single: "single"; readonly aggregate: "aggregate"};
export type SignatureSetType = typeof SignatureSetType[keyof typeof SignatureSetType];

/** a cached validator index, a PublicKey tagged with its index, or uncompressed key bytes */
export type PubkeyRef = number | {index: number} | {toBytes(compressed?: boolean): Uint8Array} | Uint8Array;

export interface ISingleSignatureSet {
  type: "single";
  pubkey: PubkeyRef;
  signingRoot: Uint8Array; // 32 bytes
  signature: Uint8Array; // 96 bytes compressed G2 (untrusted)
}
export interface IAggregatedSignatureSet {
  type: "aggregate";
  pubkeys: PubkeyRef[];
  signingRoot: Uint8Array;
  signature: Uint8Array;
}
export type ISignatureSet = ISingleSignatureSet | IAggregatedSignatureSet;

export interface BlsGpuVerifierOpts {
  devices?: number[];
  maxBufferedSigs?: number;
  maxBufferWaitMs?: number;
  blsVerifyAllMultiThread?: boolean;
  /** called once per uploaded run that held undecodable keys (those indices stay unusable) */
  onPubkeyError?: (e: Error, first: number, n: number) => void;
}

export interface BlsGpuVerifierModules {
  metrics?: unknown | null;
}

export declare class QueueError extends Error {
  type: {code: string};
}

export declare class BlsGpuVerifier implements IBlsVerifier {
  constructor(opts?: BlsGpuVerifierOpts, modules?: BlsGpuVerifierModules);
  verifySignatureSets(sets: ISignatureSet[], opts?: VerifySignatureOpts): Promise<boolean>;
  close(): Promise<void>;
  /** state-transition pubkey-added hook: (index, 48-byte pubkey, PublicKey?) */
  pubkeyAddedHook(): (index: number, pubkey: Uint8Array, pk?: object) => void;
  /** uploads the queued keys off the event loop; verifySignatureSets awaits it */
  flushPubkeys(): Promise<void>;
  onPubkeyError: ((e: Error, first: number, n: number) => void) | null;
  isValidBlsAggregate(publicKeys: PubkeyRef[], message: Uint8Array, signature: Uint8Array): Promise<boolean>;
  aggregateSignatures(sigs: Uint8Array[]): Uint8Array;
  aggregateSignaturesMany(aggregates: Uint8Array[][]): Uint8Array[];
  validatePubkeys(keys48: Uint8Array[]): (string | null)[];
  verifyDeposits(deposits: {pubkey: Uint8Array; signingRoot: Uint8Array; signature: Uint8Array}[]): boolean[];
}

/** IChainOptions fields added beside blsVerifyAllMainThread / blsVerifyAllMultiThread (options.ts:12-13) */
export interface BlsGpuChainOptions {
  blsGpu?: boolean;
  blsGpuDevices?: number[];
  blsGpuMaxBufferedSigs?: number;
  blsGpuMaxBufferWaitMs?: number;
}
export interface BlsChainOptions extends BlsGpuChainOptions {
  blsVerifyAllMainThread?: boolean;
  blsVerifyAllMultiThread?: boolean;
}

export declare const blsGpuChainOptionDefaults: Readonly<BlsGpuChainOptions>;
export declare const blsGpuCliOptions: Readonly<Record<string, object>>;
export declare function parseBlsGpuArgs(args: Record<string, unknown>): BlsGpuChainOptions;

export interface BlsVerifierImpls {
  BlsSingleThreadVerifier?: new (modules: {metrics?: unknown | null}) => IBlsVerifier;
  BlsMultiThreadWorkerPool?: new (opts: BlsChainOptions, modules: {metrics?: unknown; logger?: unknown}) => IBlsVerifier;
  setPubkeyAddedHook?: (hook: (index: number, pubkey: Uint8Array, pk?: object) => void) => void;
}

/** chain.ts:189-192 with the GPU branch */
export declare function createBlsVerifier(
  opts: BlsChainOptions,
  modules: {metrics?: unknown | null; logger?: unknown},
  impls?: BlsVerifierImpls
): IBlsVerifier;
export declare function createBlsGpuVerifier(
  opts: BlsChainOptions,
  modules?: {metrics?: unknown | null},
  setPubkeyAddedHook?: BlsVerifierImpls["setPubkeyAddedHook"]
): BlsGpuVerifier;

export declare function chunkifyMaximizeChunkSize<T>(arr: T[], minPerChunk: number): T[][];
