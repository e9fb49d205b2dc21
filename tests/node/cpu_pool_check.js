"use strict";
// CPU check of the gossip bench's CPU row (tests/test_node_cpu_pool.py): CpuPoolVerifier over the
// committed signature goldens -- every single-set batchable job concurrently (buffer flushes at
// 33 sets and on the 100 ms timer), a corrupted copy of each fourth set, and non-batchable jobs.
// Prints one JSON line {ok, checked}.
const fs = require("fs");
const path = require("path");
const {CpuPoolVerifier, loadAddon} = require(path.join(__dirname, "CpuPoolVerifier.js"));

const G = path.join(__dirname, "..", "golden");
const keys = JSON.parse(fs.readFileSync(path.join(G, "keys.json")));
const cases = JSON.parse(fs.readFileSync(path.join(G, "signatures.json"))).cases;
const hex = (s) => Uint8Array.from(Buffer.from(s, "hex"));

async function main() {
  const cpu = loadAddon();
  const pubkeys96 = new Uint8Array(96 * keys.pk_uncompressed.length);
  keys.pk_uncompressed.forEach((h, i) => pubkeys96.set(hex(h), 96 * i));
  const v = new CpuPoolVerifier({cpu, pubkeys96, workers: 4});
  const calls = [];
  cases.forEach((c, i) => {
    const set = {type: "single", pubkey: c.key, signingRoot: hex(c.msg), signature: hex(c.sig)};
    calls.push(v.verifySignatureSets([set], {batchable: true}).then((r) => r === true));
    if (i % 4 === 0) {
      const bad = hex(c.msg);
      bad[0] ^= 1;
      calls.push(v.verifySignatureSets([{...set, signingRoot: bad}], {batchable: true}).then((r) => r === false));
    }
    if (i % 8 === 1) calls.push(v.verifySignatureSets([set], {batchable: false}).then((r) => r === true));
  });
  const res = await Promise.all(calls);
  process.stdout.write(JSON.stringify({ok: res.every(Boolean), checked: res.length}) + "\n");
}

main().catch((e) => {
  process.stderr.write(String(e && e.stack) + "\n");
  process.exit(1);
});
