"use strict";
/**
 * GpuBlsVerifier: Lodestar's IBlsVerifier (beacon-node/src/chain/bls/interface.ts:20-46)
 * on the MI355X verifier, through the N-API addon integration/napi/lodestar_bls_napi.c.
 * Drop-in for BlsMultiThreadWorkerPool (multithread/index.ts): same buffering
 * (batchable jobs wait <= 100 ms or until > 32 signatures), same 128-set job split
 * (chunkifyMaximizeChunkSize), same per-call verdict / rejection semantics; GPU
 * contexts (one HIP stream each) take the place of worker threads.
 *
 * A signature set is {pubkeyIndices: number[]} (indices into the device pubkey
 * table loaded with loadPubkeys, i.e. index2pubkey) or {pubkey: Uint8Array(96)}
 * (uncompressed affine, the worker wire format of index.ts:126), plus
 * {signingRoot: Uint8Array(32), signature: Uint8Array}.
 * Plain CommonJS so it runs on the Node in this image (v12); the TypeScript
 * version is the same code with the reference's types.
 */
const path = require("path");

const addon = require(path.join(__dirname, "..", "..", "lodestar_amd", "_native", "lodestar_bls.node"));

const MAX_SIGNATURE_SETS_PER_JOB = 128; // multithread/index.ts:39
const MAX_BUFFERED_SIGS = 32; // multithread/index.ts:48
const MAX_BUFFER_WAIT_MS = 100; // multithread/index.ts:57

const ERROR_MESSAGES = {
  1: "BLST_ERROR: BLST_BAD_ENCODING",
  2: "BLST_ERROR: BLST_POINT_NOT_ON_CURVE",
  3: "BLST_ERROR: BLST_POINT_NOT_IN_GROUP",
  6: "BLST_ERROR: BLST_PK_IS_INFINITY",
  8: "BLST_ERROR: BLST_INVALID_SIZE",
  9: "ZERO_SIGNATURE",
  10: "Empty signature set",
  11: "EMPTY_AGGREGATE_ARRAY",
};

/** multithread/utils.ts:4-19 */
function chunkifyMaximizeChunkSize(arr, minPerChunk) {
  const chunkCount = Math.floor(arr.length / minPerChunk);
  if (chunkCount <= 1) return [arr];
  const perChunk = Math.ceil(arr.length / chunkCount);
  const out = [];
  for (let i = 0; i < arr.length; i += perChunk) out.push(arr.slice(i, i + perChunk));
  return out;
}

/** Pack BlsWorkReq-like jobs ({batchable, sets}) into the SoA request of bls_gpu_verify. */
function packRequests(jobs) {
  const nReq = jobs.length;
  let nSets = 0;
  for (const j of jobs) nSets += j.sets.length;
  const reqSetOffsets = new Uint32Array(nReq + 1);
  const reqBatchable = new Uint8Array(Math.max(nReq, 1));
  const messages = Buffer.alloc(Math.max(32 * nSets, 1));
  const signatures = Buffer.alloc(Math.max(96 * nSets, 1));
  const lens = new Uint32Array(Math.max(nSets, 1));
  const raw = nSets > 0 && jobs.some((j) => j.sets.some((s) => s.pubkey !== undefined));
  const pubkeys = raw ? Buffer.alloc(96 * nSets) : null;
  const setPkOffsets = raw ? null : new Uint32Array(nSets + 1);
  const idx = [];
  let k = 0;
  let anyShort = false;
  jobs.forEach((j, r) => {
    reqBatchable[r] = j.batchable ? 1 : 0;
    for (const s of j.sets) {
      Buffer.from(s.signingRoot).copy(messages, 32 * k);
      const sig = Buffer.from(s.signature);
      sig.copy(signatures, 96 * k, 0, Math.min(96, sig.length));
      lens[k] = sig.length;
      if (sig.length !== 96) anyShort = true;
      if (raw) {
        if (s.pubkey === undefined) throw Error("mixed raw / table pubkeys in one call");
        Buffer.from(s.pubkey).copy(pubkeys, 96 * k);
      } else {
        for (const i of s.pubkeyIndices) idx.push(i);
        setPkOffsets[k + 1] = idx.length;
      }
      k++;
    }
    reqSetOffsets[r + 1] = k;
  });
  return {
    reqSetOffsets,
    reqBatchable,
    messages,
    signatures,
    signatureLens: anyShort ? lens : null,
    pubkeys,
    setPkOffsets,
    pkIndices: raw ? null : Uint32Array.from(idx.length ? idx : [0]),
    seed: null,
  };
}

class GpuBlsVerifier {
  constructor(opts = {}) {
    const device = opts.device || 0;
    const contexts = opts.contexts || 2;
    this.blsVerifyAllMultiThread = Boolean(opts.blsVerifyAllMultiThread);
    this.maxSetsPerCall = opts.maxSetsPerCall || MAX_SIGNATURE_SETS_PER_JOB;
    this.ctxs = [];
    for (let i = 0; i < contexts; i++) this.ctxs.push({handle: addon.init(device), busy: false});
    this.jobs = [];
    this.bufferedJobs = null;
    this.closed = false;
    this.metrics = {jobsStarted: 0, sigSetsStarted: 0};
  }

  /** Append validator pubkeys (48 B compressed each) to every context's device table. */
  loadPubkeys(pks48) {
    for (const c of this.ctxs) {
      const codes = addon.loadPubkeys(c.handle, pks48, 48);
      const bad = codes.findIndex((x) => x !== 0);
      if (bad >= 0) throw Error(`invalid pubkey at index ${bad}`);
    }
  }

  /** IBlsVerifier.verifySignatureSets (index.ts:134-174) */
  async verifySignatureSets(sets, opts = {}) {
    if (opts.verifyOnMainThread && !this.blsVerifyAllMultiThread) {
      // "don't buffer": one non-batchable request now (verifySignatureSetsMaybeBatch)
      return this._settle(await this._call(this.ctxs[0], [{batchable: false, sets}]), 0);
    }
    const results = await Promise.all(
      chunkifyMaximizeChunkSize(sets, MAX_SIGNATURE_SETS_PER_JOB).map((chunk) =>
        this._queue({batchable: Boolean(opts.batchable), sets: chunk})
      )
    );
    if (results.length === 0) throw Error("Empty results array");
    return results.every((v) => v === true);
  }

  /** IBlsVerifier.close (index.ts:176-197) */
  async close() {
    this.closed = true;
    if (this.bufferedJobs) clearTimeout(this.bufferedJobs.timeout);
    const pending = this.jobs.concat(this.bufferedJobs ? this.bufferedJobs.jobs : []);
    this.jobs = [];
    this.bufferedJobs = null;
    for (const j of pending) j.reject(Error("QUEUE_ABORTED"));
    while (this.ctxs.some((c) => c.busy)) await new Promise((r) => setTimeout(r, 5));
    for (const c of this.ctxs) addon.close(c.handle);
    this.ctxs = [];
  }

  _settle(verdicts, i) {
    const code = verdicts[i];
    if (code < 0) throw Error(ERROR_MESSAGES[-code] || `BLST_ERROR: ${-code}`);
    return code === 1;
  }

  async _call(ctx, jobs) {
    ctx.busy = true;
    try {
      return await addon.verify(ctx.handle, packRequests(jobs));
    } finally {
      ctx.busy = false;
    }
  }

  /** queueBlsWork (index.ts:238-285) */
  _queue(workReq) {
    if (this.closed) return Promise.reject(Error("QUEUE_ABORTED"));
    return new Promise((resolve, reject) => {
      const job = {resolve, reject, workReq, addedTimeMs: Date.now()};
      if (workReq.batchable) {
        if (!this.bufferedJobs) {
          this.bufferedJobs = {jobs: [], sigCount: 0, timeout: setTimeout(() => this._runBufferedJobs(), MAX_BUFFER_WAIT_MS)};
        }
        this.bufferedJobs.jobs.push(job);
        this.bufferedJobs.sigCount += workReq.sets.length;
        if (this.bufferedJobs.sigCount > MAX_BUFFERED_SIGS) {
          clearTimeout(this.bufferedJobs.timeout);
          this._runBufferedJobs();
        }
      } else {
        this.jobs.push(job);
        setTimeout(() => this._runJob(), 0);
      }
    });
  }

  _runBufferedJobs() {
    if (this.bufferedJobs) {
      this.jobs.push(...this.bufferedJobs.jobs);
      this.bufferedJobs = null;
      setTimeout(() => this._runJob(), 0);
    }
  }

  /** runJob / prepareWork (index.ts:290-400) with GPU contexts as the workers */
  async _runJob() {
    if (this.closed) return;
    const ctx = this.ctxs.find((c) => !c.busy);
    if (!ctx || this.jobs.length === 0) return;
    const jobs = [];
    let total = 0;
    while (total < this.maxSetsPerCall && this.jobs.length > 0) {
      const j = this.jobs.shift();
      jobs.push(j);
      total += j.workReq.sets.length;
    }
    this.metrics.jobsStarted += jobs.length;
    this.metrics.sigSetsStarted += total;
    let verdicts;
    try {
      verdicts = await this._call(ctx, jobs.map((j) => j.workReq));
    } catch (e) {
      for (const j of jobs) j.reject(e);
      setTimeout(() => this._runJob(), 0);
      return;
    }
    jobs.forEach((j, i) => {
      try {
        j.resolve(this._settle(verdicts, i));
      } catch (e) {
        j.reject(e);
      }
    });
    setTimeout(() => this._runJob(), 0);
  }
}

module.exports = {GpuBlsVerifier, chunkifyMaximizeChunkSize, packRequests, ERROR_MESSAGES};
