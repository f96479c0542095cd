"use strict";
/** Host-side test of GpuBlsVerifier's queueing with a stand-in addon (tests/test_napi.py). */
const {GpuBlsVerifier} = require("./gpuBlsVerifier.js");

async function main() {
  const calls = [];
  const rawCalls = [];
  const handles = [];
  let inflight = 0;
  const fake = {
    init: (dev, high) => {
      const h = {high: Boolean(high), calls: 0};
      handles.push(h);
      return h;
    },
    close: () => {},
    loadPubkeys: () => new Int32Array(0),
    verify: (h, req) => {
      const n = req.reqSetOffsets.length - 1;
      h.calls++;
      (req.pubkeys ? rawCalls : calls).push(req.reqSetOffsets[n]);
      inflight++;
      const t0 = Number(process.hrtime.bigint());
      return new Promise((res) =>
        setTimeout(() => {
          inflight--;
          const v = new Int32Array(n);
          let ok = 0;
          for (let r = 0; r < n; r++) {
            const k = req.reqSetOffsets[r];
            v[r] = req.signatureLens && req.signatureLens[k] !== 96 ? -8 : req.signingRoot === undefined ? req.messages[32 * k] & 1 : 1;
            if (v[r] === 1) ok += req.reqSetOffsets[r + 1] - k;
          }
          // the addon's BlsWorkResult bookkeeping (lodestar_bls_napi.c attach_stats)
          v.batchRetries = v.some((x) => x !== 1) ? 1 : 0;
          v.batchSigsSuccess = ok;
          v.workerStartNs = t0 + 1e5;
          v.workerEndNs = Number(process.hrtime.bigint()) - 1e5;
          res(v);
        }, 5)
      );
    },
  };
  // stand-in prom-client metrics with the reference's names (lodestar.ts:378-446)
  const seen = {};
  const metric = (name) => ({
    inc: (a, b) => { seen[name] = (seen[name] || 0) + (typeof a === "number" ? a : b); },
    observe: (x) => { seen[name] = (seen[name] || 0) + 1; if (!(x >= 0)) seen[name + "_bad"] = x; },
    set: (x) => { seen[name] = x; },
    startTimer: () => () => { seen[name] = (seen[name] || 0) + 1; },
    addCollect: (fn) => { seen.collect = fn; },
  });
  const metrics = {bls: {aggregatedPubkeys: metric("aggregatedPubkeys")}, blsThreadPool: {}};
  for (const k of ["jobsWorkerTime", "jobWaitTime", "latencyToWorker", "latencyFromWorker", "batchRetries",
                   "batchSigsSuccess", "queueLength", "totalJobsGroupsStarted", "totalJobsStarted", "totalSigSetsStarted",
                   "successJobsSignatureSetsCount", "errorJobsSignatureSetsCount", "mainThreadDurationInThreadPool"])
    metrics.blsThreadPool[k] = metric(k);
  const pool = new GpuBlsVerifier({contexts: 2, addon: fake, metrics});
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
  // the five series the reference feeds from BlsWorkResult (index.ts:130,357-366)
  seen.collect();
  out.series = ["batchRetries", "batchSigsSuccess", "latencyToWorker", "latencyFromWorker"].map((k) => seen[k] || 0);
  out.series_bad = Object.keys(seen).filter((k) => k.endsWith("_bad"));
  out.queue_length_metric = typeof seen.queueLength === "number";
  out.stats_retries = pool.stats.batchRetries;
  // raw-key jobs: calls of one worker message (prepareWork: jobs until >= 128 sets)
  const raw = [];
  for (let i = 0; i < 300; i++) raw.push(pool.verifySignatureSets([{pubkey: Buffer.alloc(96, 1), signingRoot: Buffer.alloc(32, 1), signature: Buffer.alloc(96, 1)}], {batchable: true}));
  await Promise.all(raw);
  out.raw_max_call_sets = Math.max(...rawCalls);
  // the main-thread lane: its own high-priority context, never a pool context
  const mainBefore = handles.filter((h) => h.high).map((h) => h.calls);
  await pool.verifySignatureSets([sets[1]], {verifyOnMainThread: true});
  out.main_handles = handles.filter((h) => h.high).length;
  out.main_calls = handles.filter((h) => h.high).map((h) => h.calls - mainBefore.shift());
  out.pool_high = handles.filter((h) => !h.high).length;
  const queued = [];
  for (let i = 0; i < 2000; i++) queued.push(pool.verifySignatureSets([sets[i]], {batchable: true}).then(() => "resolved", (e) => e.message));
  await new Promise((r) => setTimeout(r, 1));
  await pool.close();
  out.inflight_at_close = inflight;
  const q = await Promise.all(queued);
  out.closed = q.find((x) => x !== "resolved" && x !== true) || "none";
  // libuv pool warning against a stand-in pool of 4 threads (3 contexts + 2 > 4)
  const warnings = [];
  const w = new GpuBlsVerifier({contexts: 3, addon: fake, uvThreadpoolSize: 4, warn: (m) => warnings.push(m)});
  await w.close();
  out.pool_warning = warnings[0] || null;
  // scratch admission: the library refuses pool contexts past its budget (BLS_ERR_ADMISSION)
  const refusing = (admit) => Object.assign({}, fake, {
    init: (dev, high) => {
      if (!high && admit-- <= 0) {
        const e = Error("BLS_ERR_ADMISSION: stand-in refusal");
        e.code = "BLS_ERR_ADMISSION";
        throw e;
      }
      return fake.init(dev, high);
    },
  });
  const part = new GpuBlsVerifier({contexts: 3, addon: refusing(1), uvThreadpoolSize: 64});
  out.admitted_partial = {ctxs: part.ctxs.length, errors: part.initErrors.length,
                          verdict: await part.verifySignatureSets([sets[1]], {batchable: false})};
  await part.close();
  const none = new GpuBlsVerifier({contexts: 2, addon: refusing(0), uvThreadpoolSize: 64});
  out.admitted_none = await none.verifySignatureSets([sets[1]], {batchable: true}).then(() => "resolved", (e) => e.message);
  await none.close();
  console.log(JSON.stringify(out));
}

main().catch((e) => {
  console.error(e && e.stack);
  process.exit(1);
});
