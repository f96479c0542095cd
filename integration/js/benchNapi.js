"use strict";
/**
 * bench.py --mode napi: the cfg2 workload through the N-API addon and GpuBlsVerifier,
 * driven the way gossip validation drives IBlsVerifier (setsPerCall = 1: one
 * verifySignatureSets([set], {batchable: true}) per attestation,
 * chain/validation/attestation.ts:138) or the way sync / block import does (calls of
 * setsPerCall sets, sync/range/range.ts:191-214).  A step submits inflight x nSets
 * sets; two steps are kept outstanding so the contexts never wait for the JS side.
 *
 *   node benchNapi.js work.json steps contexts nSets [setsPerCall [maxSetsPerCall [devices]]]   -> one JSON line
 * (maxSetsPerCall: sets per GPU call the adapter coalesces queued jobs into; devices: the
 * adapter's device slots, comma-separated -- "0,0" runs two slots on one GPU; `contexts`
 * is per slot)
 */
const fs = require("fs");
const {GpuBlsVerifier} = require("./gpuBlsVerifier.js");

async function main() {
  const [file, stepsS, inflightS, nSetsS] = process.argv.slice(2);
  const steps = Number(stepsS);
  const inflight = Number(inflightS);
  const nSets = Number(nSetsS);
  const perCall = Number(process.argv[6] || 1);
  const maxSetsPerCall = Number(process.argv[7] || 1024);
  const devices = String(process.argv[8] || "0").split(",").map(Number);
  const data = JSON.parse(fs.readFileSync(file, "utf8"));
  const sets = data.sets.map((s) => ({
    pubkeyIndices: [s.idx],
    signingRoot: Buffer.from(s.msg, "hex"),
    signature: Buffer.from(s.sig, "hex"),
  }));
  const pool = new GpuBlsVerifier({contexts: inflight, maxSetsPerCall, devices});
  pool.loadPubkeys(Buffer.from(data.pubkeys48, "hex"));
  const per = devices.length * inflight * nSets * Math.max(1, Math.round(maxSetsPerCall / nSets));
  const calls = [];
  for (let k = 0; k < per; k += perCall) {
    const c = [];
    for (let j = k; j < Math.min(per, k + perCall); j++) c.push(sets[j % nSets]);
    calls.push(c);
  }
  const step = () => Promise.all(calls.map((c) => pool.verifySignatureSets(c, {batchable: true})));
  const check = (r) => {
    for (const v of r) if (v !== true) throw Error("a valid set did not verify");
  };
  check(await step()); // warm-up
  const cpu0 = process.cpuUsage();
  const t0 = process.hrtime.bigint();
  const pending = [];
  for (let s = 0; s < steps; s++) {
    pending.push(step());
    if (pending.length >= 2) check(await pending.shift());
  }
  for (const p of pending) check(await p);
  const dt = Number(process.hrtime.bigint() - t0) / 1e9;
  const cpu = process.cpuUsage(cpu0); // the process's CPU time over the timed steps (every thread)
  const st = pool.stats;
  await pool.close();
  console.log(JSON.stringify({sets_per_s: (steps * per) / dt, elapsed_s: dt, steps, sets_per_step: per,
                              cpu_s_per_wall_s: (cpu.user + cpu.system) / 1e6 / dt, sets_per_call: perCall, max_sets_per_gpu_call: maxSetsPerCall, contexts: inflight,
                              gpu_calls: st.jobGroupsStarted, jobs: st.jobsStarted, devices,
                              slot_sets: pool.slotStats.map((x) => x.sets)}));
}

main().catch((e) => {
  console.error("benchNapi failed:", e && e.stack);
  process.exit(1);
});
