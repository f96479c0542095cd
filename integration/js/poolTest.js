"use strict";
/**
 * The reference's pool e2e test (beacon-node/test/e2e/chain/bls/multithread.test.ts)
 * run against GpuBlsVerifier.  Input: a JSON file with {pubkeys48: hex, sets: [{idx,
 * msg, sig}]} (made by tests/test_napi.py).  Prints one JSON line of results.
 */
const fs = require("fs");
const assert = require("assert");
const {GpuBlsVerifier, chunkifyMaximizeChunkSize} = require("./gpuBlsVerifier.js");

async function main() {
  const data = JSON.parse(fs.readFileSync(process.argv[2], "utf8"));
  const sets = data.sets.map((s) => ({
    pubkeyIndices: [s.idx],
    signingRoot: Buffer.from(s.msg, "hex"),
    signature: Buffer.from(s.sig, "hex"),
  }));
  const pool = new GpuBlsVerifier({contexts: 2});
  pool.loadPubkeys(Buffer.from(data.pubkeys48, "hex"));
  const out = {};

  // utils.test.ts (KAT-5)
  out.chunkify = [1, 2, 3, 4, 5, 6, 7, 8].map((n) => chunkifyMaximizeChunkSize([...Array(n).keys()], 3));

  for (const [name, opts, sleep] of [
    ["sync", {}, false],
    ["async", {}, true],
    ["batched", {batchable: true}, true],
    ["mainThread", {verifyOnMainThread: true}, false],
  ]) {
    const ps = [];
    for (let i = 0; i < 8; i++) {
      ps.push(pool.verifySignatureSets(sets, opts));
      if (sleep) await new Promise((r) => setTimeout(r, 5));
    }
    out[name] = await Promise.all(ps);
  }

  // "Should verify multiple signatures batched, first is invalid"
  const invalid = Object.assign({}, sets[0], {signature: Buffer.alloc(32, 0)});
  const bad = pool.verifySignatureSets([invalid], {batchable: true}).then(
    () => "resolved",
    (e) => e.message
  );
  const good = [];
  for (let i = 0; i < 8; i++) good.push(pool.verifySignatureSets(sets, {batchable: true}));
  out.firstInvalid = await bad;
  out.firstInvalidOthers = await Promise.all(good);

  const wrong = Object.assign({}, sets[1], {signingRoot: sets[0].signingRoot});
  out.wrongMessage = await pool.verifySignatureSets(sets.concat([wrong]));
  out.empty = await pool.verifySignatureSets([]).then(() => "resolved", (e) => e.message);
  // state-transition verifySignatureSet, synchronous (signatureSets.ts:24-38)
  out.stfSync = [sets[0], wrong, invalid].map((s) => {
    try {
      return pool.verifySignatureSetSync(s);
    } catch (e) {
      return e.message;
    }
  });
  const each = pool.verifySignatureSetsEachSync([sets[0], wrong, sets[2], invalid]);
  out.stfEach = each.map((r) => r.valid);
  // an undecodable set is never truthy (ADVICE r3: a mixed boolean / Error array was)
  out.stfEachInvalid = [Boolean(each[3].valid), each[3].error ? each[3].error.message : null];
  await pool.close();
  assert.ok(true);
  console.log(JSON.stringify(out));
}

main().catch((e) => {
  console.error("poolTest failed:", e && e.message, e && e.stack);
  process.exit(1);
});
