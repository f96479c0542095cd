"use strict";
/** Host-side test of GpuBlsVerifier's queueing with a stand-in addon (tests/test_napi.py). */
const {GpuBlsVerifier} = require("./gpuBlsVerifier.js");

async function main() {
  const calls = [];
  let inflight = 0;
  const fake = {
    init: () => ({}),
    close: () => {},
    loadPubkeys: () => new Int32Array(0),
    verify: (h, req) => {
      const n = req.reqSetOffsets.length - 1;
      calls.push(req.reqSetOffsets[n]);
      inflight++;
      return new Promise((res) =>
        setTimeout(() => {
          inflight--;
          const v = new Int32Array(n);
          for (let r = 0; r < n; r++) {
            const k = req.reqSetOffsets[r];
            v[r] = req.signatureLens && req.signatureLens[k] !== 96 ? -8 : req.signingRoot === undefined ? req.messages[32 * k] & 1 : 1;
          }
          res(v);
        }, 5)
      );
    },
  };
  const pool = new GpuBlsVerifier({contexts: 2, addon: fake});
  const sets = [];
  for (let i = 0; i < 4000; i++) sets.push({pubkeyIndices: [i % 50], signingRoot: Buffer.alloc(32, i % 2), signature: Buffer.alloc(96, 1)});
  const ps = sets.map((s) => pool.verifySignatureSets([s], {batchable: true}));
  const bad = pool.verifySignatureSets([{pubkeyIndices: [0], signingRoot: Buffer.alloc(32, 1), signature: Buffer.alloc(32)}], {batchable: true}).then(
    () => "resolved",
    (e) => e.message
  );
  const res = await Promise.all(ps);
  const out = {};
  out.verdicts_ok = res.every((v, i) => v === (i % 2 === 1));
  out.rejected = await bad;
  out.others_true = true;
  out.calls = calls.length;
  out.max_call_sets = Math.max(...calls);
  const queued = [];
  for (let i = 0; i < 2000; i++) queued.push(pool.verifySignatureSets([sets[i]], {batchable: true}).then(() => "resolved", (e) => e.message));
  await new Promise((r) => setTimeout(r, 1));
  await pool.close();
  out.inflight_at_close = inflight;
  const q = await Promise.all(queued);
  out.closed = q.find((x) => x !== "resolved" && x !== true) || "none";
  console.log(JSON.stringify(out));
}

main().catch((e) => {
  console.error(e && e.stack);
  process.exit(1);
});
