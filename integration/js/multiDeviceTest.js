"use strict";
/**
 * GpuBlsVerifier over several device slots (one verifier per node; VERDICT r5 item 1):
 * routing of per-set gossip calls to the least-loaded slot, and the split of one large
 * non-batchable call across the slots (addon.partial per slot, one addon.finalCheck).
 *
 *   node multiDeviceTest.js work.json     -> the real addon, devices [0, 0] (tests/test_napi.py, GPU)
 *   node multiDeviceTest.js --stand-in    -> a stand-in addon over validity tokens (host logic, CPU)
 *
 * work.json: {pubkeys48: hex, sets: [{idx, msg, sig}]} of >= 512 valid sets.  Prints one
 * JSON line of results.
 */
const fs = require("fs");
const {GpuBlsVerifier} = require("./gpuBlsVerifier.js");

/** A stand-in addon: a set's signature byte 0 is 1 (valid) or 0 (invalid); a partial
 * carries its shard's count of invalid sets; a signature of another length does not
 * decode (status -8). */
function standIn() {
  const calls = [];
  const verdictOf = (req, r) => {
    for (let k = req.reqSetOffsets[r]; k < req.reqSetOffsets[r + 1]; k++) {
      if (req.signatureLens && req.signatureLens[k] !== 96) return -8;
    }
    for (let k = req.reqSetOffsets[r]; k < req.reqSetOffsets[r + 1]; k++) if (req.signatures[96 * k] !== 1) return 0;
    return 1;
  };
  const later = (v) => new Promise((res) => setTimeout(() => res(v), 2));
  return {
    calls,
    init: (dev, high) => ({dev, high}),
    close: () => {},
    loadPubkeys: () => new Int32Array(0),
    verify: (h, req) => {
      const n = req.reqSetOffsets.length - 1;
      calls.push({kind: "verify", dev: h.dev, sets: req.reqSetOffsets[n]});
      const v = new Int32Array(n);
      for (let r = 0; r < n; r++) v[r] = verdictOf(req, r);
      v.batchRetries = 0;
      v.batchSigsSuccess = 0;
      return later(v);
    },
    partial: (h, req, base) => {
      const n = req.reqSetOffsets[req.reqSetOffsets.length - 1];
      calls.push({kind: "partial", dev: h.dev, sets: n, base, seed: Buffer.from(req.seed).toString("hex")});
      let bad = 0;
      for (let k = 0; k < n; k++) {
        if (req.signatureLens && req.signatureLens[k] !== 96) return later({partial: null, status: -8, errClass: 1, errIndex: k});
        if (req.signatures[96 * k] !== 1) bad++;
      }
      const p = new Uint8Array(576);
      p[0] = bad;
      return later({partial: p, status: 0, errClass: 3, errIndex: 0});
    },
    finalCheck: (h, parts) => {
      calls.push({kind: "final", dev: h.dev, n: parts.length / 576});
      let bad = 0;
      for (let k = 0; k < parts.length; k += 576) bad += parts[k];
      return later(bad === 0);
    },
  };
}

async function main() {
  const stand = process.argv[2] === "--stand-in";
  let sets;
  let pks = null;
  const fake = stand ? standIn() : null;
  const tamper = (s) => stand
    ? Object.assign({}, s, {signature: Buffer.alloc(96, 0)})
    : Object.assign({}, s, {signingRoot: Buffer.from(s.signingRoot.map((b) => b ^ 0xff))});
  if (stand) {
    sets = [];
    for (let i = 0; i < 512; i++) sets.push({pubkeyIndices: [i], signingRoot: Buffer.alloc(32, i & 255), signature: Buffer.alloc(96, 1)});
  } else {
    const data = JSON.parse(fs.readFileSync(process.argv[2], "utf8"));
    pks = Buffer.from(data.pubkeys48, "hex");
    sets = data.sets.map((s) => ({pubkeyIndices: [s.idx], signingRoot: Buffer.from(s.msg, "hex"), signature: Buffer.from(s.sig, "hex")}));
  }
  const pool = new GpuBlsVerifier({devices: [0, 0], contexts: 2, splitCallMinSets: 256, addon: fake || undefined, maxSetsPerCall: 128,
                                   uvThreadpoolSize: 64});
  if (pks) pool.loadPubkeys(pks);
  const out = {slots: pool.slotCtxs.map((c) => c.length)};
  // routing: per-set batchable calls, 5 invalid
  const bad = new Set([5, 77, 300, 301, 450]);
  const gossip = sets.map((s, i) => (bad.has(i) ? tamper(s) : s));
  const v = await Promise.all(gossip.map((s) => pool.verifySignatureSets([s], {batchable: true})));
  out.gossipOk = v.every((x, i) => x === !bad.has(i));
  out.slotSets = pool.slotStats.map((x) => x.sets);
  // the split call
  out.splitValid = await pool.verifySignatureSets(sets);
  const one = sets.slice();
  one[400] = tamper(one[400]);
  out.splitInvalid = await pool.verifySignatureSets(one);
  out.badShards = pool.splitStats.badShards;
  const short = sets.slice();
  short[10] = tamper(short[10]);
  short[300] = Object.assign({}, short[300], {signature: Buffer.alloc(32)});
  out.splitError = await pool.verifySignatureSets(short).then(() => "resolved", (e) => e.message);
  out.splitStats = pool.splitStats;
  // batchable: not split
  out.batchableValid = await pool.verifySignatureSets(sets, {batchable: true});
  out.splitCallsAfterBatchable = pool.splitStats.calls;
  if (fake) {
    const parts = fake.calls.filter((c) => c.kind === "partial");
    out.partials = parts.slice(0, 2).map((c) => [c.base, c.sets]);
    out.sharedSeed = parts.length >= 2 && parts[0].seed === parts[1].seed;
    out.finals = fake.calls.filter((c) => c.kind === "final").map((c) => c.n);
  }
  await pool.close();
  console.log(JSON.stringify(out));
}

main().catch((e) => {
  console.error(e && e.stack);
  process.exit(1);
});
