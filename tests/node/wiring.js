"use strict";
// Loads the package entry of lodestar_amd/node and checks the verifier selection of
// chain.ts:189-192 with the GPU branch, and the chain-option / CLI-flag parsing.
// CPU-only (stand-in CPU verifiers; the GPU branch is taken only with BGV_WIRING_GPU=1,
// where it verifies one signature set on the device: tests/test_node_wiring.py).
const assert = require("assert");
const path = require("path");
const pkg = require(path.join(__dirname, "..", "..", "lodestar_amd", "node"));

class FakeSingle {
  constructor(modules) {
    this.kind = "single";
    this.modules = modules;
  }
}
class FakePool {
  constructor(opts, modules) {
    this.kind = "pool";
    this.opts = opts;
  }
}
const impls = {BlsSingleThreadVerifier: FakeSingle, BlsMultiThreadWorkerPool: FakePool};

(async () => {
  // selection order: main thread first, then GPU, then the worker pool
  assert.strictEqual(pkg.createBlsVerifier({blsVerifyAllMainThread: true, blsGpu: true}, {}, impls).kind, "single");
  assert.strictEqual(pkg.createBlsVerifier({}, {}, impls).kind, "pool");
  assert.strictEqual(pkg.createBlsVerifier({...pkg.blsGpuChainOptionDefaults}, {}, impls).kind, "pool");
  assert.throws(() => pkg.createBlsVerifier({}, {}, {}), /BlsMultiThreadWorkerPool not provided/);

  // CLI -> options
  const o = pkg.parseBlsGpuArgs({"chain.blsGpu": true, "chain.blsGpuDevices": ["0", "3"], "chain.blsGpuMaxBufferWaitMs": 2});
  assert.deepStrictEqual(o, {blsGpu: true, blsGpuDevices: [0, 3], blsGpuMaxBufferedSigs: undefined, blsGpuMaxBufferWaitMs: 2});
  assert.deepStrictEqual(pkg.parseBlsGpuArgs({"chain.blsGpuDevices": "1,2"}).blsGpuDevices, [1, 2]);
  assert.throws(() => pkg.parseBlsGpuArgs({"chain.blsGpuDevices": ["-1"]}), /Invalid --chain.blsGpuDevices/);
  for (const k of ["chain.blsGpu", "chain.blsGpuDevices", "chain.blsGpuMaxBufferedSigs", "chain.blsGpuMaxBufferWaitMs"]) {
    assert.ok(pkg.blsGpuCliOptions[k] && pkg.blsGpuCliOptions[k].group === "chain", k);
  }
  assert.strictEqual(pkg.blsGpuChainOptionDefaults.blsGpu, false);

  if (process.env.BGV_WIRING_GPU === "1") {
    let hook = null;
    const v = pkg.createBlsVerifier({blsGpu: true, blsGpuDevices: [0]}, {metrics: null}, {
      ...impls,
      setPubkeyAddedHook: (h) => (hook = h),
    });
    assert.ok(v instanceof pkg.BlsGpuVerifier, "GPU branch builds BlsGpuVerifier");
    assert.strictEqual(typeof hook, "function", "pubkey hook installed");
    const gold = require(path.join(__dirname, "..", "golden", "keys.json"));
    const sigs = require(path.join(__dirname, "..", "golden", "signatures.json"));
    const hex = (h) => Uint8Array.from(Buffer.from(h, "hex"));
    // validator 0's compressed key through the hook, then one set by index
    hook(0, hex(gold.pk_compressed[0]), {});
    const s = sigs.cases.find((x) => x.key === 0);
    const ok = await v.verifySignatureSets([{type: "single", pubkey: 0, signingRoot: hex(s.msg), signature: hex(s.sig)}]);
    assert.strictEqual(ok, true);
    const bad = await v.verifySignatureSets([{type: "single", pubkey: 0, signingRoot: hex(s.msg).map((b, i) => (i ? b : b ^ 1)),
      signature: hex(s.sig)}]);
    assert.strictEqual(bad, false);
    await v.close();
  }
  console.log("wiring ok");
})().catch((e) => {
  console.error(e);
  process.exit(1);
});
