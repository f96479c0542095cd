"use strict";
/**
 * verifyOnMainThread while the pool is busy (multithread/index.ts:138-151: the reference
 * runs it synchronously on the main thread, outside the worker queue).  The adapter
 * sends it to its own high-priority context, so it must not wait for a large pool call
 * in flight.  Input: {pubkeys48: hex, sets: [{idx, msg, sig}]} (tests/test_napi.py);
 * prints one JSON line: the main-thread call's latency, the pool call's, and their order.
 */
const fs = require("fs");
const {GpuBlsVerifier} = require("./gpuBlsVerifier.js");

const now = () => Number(process.hrtime.bigint()) / 1e6;

async function main() {
  const data = JSON.parse(fs.readFileSync(process.argv[2], "utf8"));
  const sets = data.sets.map((s) => ({
    pubkeyIndices: [s.idx],
    signingRoot: Buffer.from(s.msg, "hex"),
    signature: Buffer.from(s.sig, "hex"),
  }));
  const v = new GpuBlsVerifier({contexts: 1, maxSetsPerCall: sets.length});
  v.loadPubkeys(Buffer.from(data.pubkeys48, "hex"));
  // warm-up: both lanes once
  await v.verifySignatureSets(sets.slice(0, 256), {batchable: true});
  await v.verifySignatureSets([sets[0]], {verifyOnMainThread: true});
  const out = {runs: []};
  for (let rep = 0; rep < 3; rep++) {
    const t0 = now();
    let poolDone = 0;
    const pool = v.verifySignatureSets(sets, {batchable: true}).then((ok) => {
      poolDone = now();
      return ok;
    });
    await new Promise((r) => setTimeout(r, 2));  // the pool call is on the GPU
    const t1 = now();
    const main = await v.verifySignatureSets([sets[rep + 1]], {verifyOnMainThread: true});
    const t2 = now();
    const poolOk = await pool;
    out.runs.push({main_ok: main, pool_ok: poolOk, main_ms: t2 - t1, pool_ms: poolDone - t0,
                   main_before_pool: poolDone === 0 || t2 < poolDone});
  }
  // the same main-thread call alone
  const t3 = now();
  await v.verifySignatureSets([sets[5]], {verifyOnMainThread: true});
  out.main_alone_ms = now() - t3;
  console.log(JSON.stringify(out));
  await v.close();
}

main().catch((e) => {
  console.error(e);
  process.exit(1);
});
