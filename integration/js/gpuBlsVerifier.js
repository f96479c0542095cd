"use strict";
/**
 * GpuBlsVerifier: Lodestar's IBlsVerifier (beacon-node/src/chain/bls/interface.ts:20-46)
 * on the MI355X verifier, through the N-API addon integration/napi/lodestar_bls_napi.c.
 * Drop-in for BlsMultiThreadWorkerPool (multithread/index.ts): same buffering
 * (batchable jobs wait <= 100 ms or until > 32 signatures), same 128-set job split
 * (chunkifyMaximizeChunkSize), same per-call verdict / rejection semantics; GPU
 * contexts (one HIP stream each) take the place of worker threads.  A context takes
 * queued jobs up to GPU_SETS_PER_CALL sets per call (the reference's 128 per worker
 * message is a CPU-core size; verdicts per job do not depend on it, worker.ts:56),
 * and feeds the reference's metric series (metrics.bls / metrics.blsThreadPool,
 * lodestar.ts:378-446) when a metrics object is passed.
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
const GPU_SETS_PER_CALL = 1024; // sets per bls_gpu_verify call (cfg2 shape)
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
      if (s.signingRoot.length !== 32) throw Error("signing roots are 32 bytes");
      messages.set(s.signingRoot, 32 * k);
      const sig = s.signature;
      signatures.set(sig.length > 96 ? sig.subarray(0, 96) : sig, 96 * k);
      lens[k] = sig.length;
      if (sig.length !== 96) anyShort = true;
      if (raw) {
        if (s.pubkey === undefined) throw Error("mixed raw / table pubkeys in one call");
        if (s.pubkey.length !== 96) throw Error("raw pubkeys are 96 bytes (uncompressed affine)");
        pubkeys.set(s.pubkey, 96 * k);
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

/** getAggregatedPubkeysCount (chain/bls/utils.ts:18-26): keys of aggregate-type sets */
function getAggregatedPubkeysCount(sets) {
  let n = 0;
  for (const s of sets) {
    const agg = s.type !== undefined ? s.type === "aggregate" : s.pubkeyIndices !== undefined && s.pubkeyIndices.length > 1;
    if (agg && s.pubkeyIndices !== undefined) n += s.pubkeyIndices.length;
  }
  return n;
}

class GpuBlsVerifier {
  constructor(opts = {}) {
    const device = opts.device || 0;
    const contexts = opts.contexts || 2;
    this.blsVerifyAllMultiThread = Boolean(opts.blsVerifyAllMultiThread);
    this.maxSetsPerCall = opts.maxSetsPerCall || GPU_SETS_PER_CALL;
    this.metrics = opts.metrics || null; // {bls: {...}, blsThreadPool: {...}} with the reference's names
    this.ctxs = [];
    // `inflight`: calls queued or running on the context (the main-thread path may
    // share context 0 with a pool job; the library serialises calls per context)
    for (let i = 0; i < contexts; i++) this.ctxs.push({handle: addon.init(device), inflight: 0, id: i});
    this.jobs = [];
    this.bufferedJobs = null;
    this.closed = false;
    this.stats = {jobsStarted: 0, sigSetsStarted: 0, jobGroupsStarted: 0, batchRetries: 0};
  }

  /** Append validator pubkeys (48 B compressed each) to every context's device table.
   * All or nothing (bls_gpu_load_pubkeys appends no key of a batch holding a bad one). */
  loadPubkeys(pks48) {
    this.ctxs.forEach((c, i) => {
      const codes = addon.loadPubkeys(c.handle, pks48, 48);
      const bad = codes.findIndex((x) => x !== 0);
      if (bad >= 0) throw Error(i === 0 ? `invalid pubkey at batch index ${bad}; no key appended` : "pubkey tables diverged");
    });
  }

  /** IBlsVerifier.verifySignatureSets (index.ts:134-174) */
  async verifySignatureSets(sets, opts = {}) {
    if (this.metrics) this.metrics.bls.aggregatedPubkeys.inc(getAggregatedPubkeysCount(sets));
    if (opts.verifyOnMainThread && !this.blsVerifyAllMultiThread) {
      // "don't buffer": one non-batchable request now (verifySignatureSetsMaybeBatch)
      const timer = this.metrics && this.metrics.blsThreadPool.mainThreadDurationInThreadPool.startTimer();
      try {
        return this._settle(await this._call(this.ctxs[0], [{batchable: false, sets}]), 0);
      } finally {
        if (timer) timer();
      }
    }
    if (sets.length > 0 && sets.length <= MAX_SIGNATURE_SETS_PER_JOB) {
      // one job (chunkifyMaximizeChunkSize gives one chunk): skip the Promise.all
      return (await this._queue({batchable: Boolean(opts.batchable), sets})) === true;
    }
    const results = await Promise.all(
      chunkifyMaximizeChunkSize(sets, MAX_SIGNATURE_SETS_PER_JOB).map((chunk) =>
        this._queue({batchable: Boolean(opts.batchable), sets: chunk})
      )
    );
    if (results.length === 0) throw Error("Empty results array");
    return results.every((v) => v === true);
  }

  /** IBlsVerifier.close (index.ts:176-197): abort queued jobs, wait for calls in flight */
  async close() {
    this.closed = true;
    if (this.bufferedJobs) clearTimeout(this.bufferedJobs.timeout);
    const pending = this.jobs.concat(this.bufferedJobs ? this.bufferedJobs.jobs : []);
    this.jobs = [];
    this.bufferedJobs = null;
    for (const j of pending) j.reject(Error("QUEUE_ABORTED"));
    while (this.ctxs.some((c) => c.inflight > 0)) await new Promise((r) => setTimeout(r, 5));
    for (const c of this.ctxs) addon.close(c.handle);
    this.ctxs = [];
  }

  _settle(verdicts, i) {
    const code = verdicts[i];
    if (code < 0) throw Error(ERROR_MESSAGES[-code] || `BLST_ERROR: ${-code}`);
    return code === 1;
  }

  async _call(ctx, jobs) {
    if (this.closed && this.ctxs.length === 0) throw Error("QUEUE_ABORTED");
    ctx.inflight++;
    try {
      return await addon.verify(ctx.handle, packRequests(jobs));
    } finally {
      ctx.inflight--;
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

  /** runJob / prepareWork (index.ts:290-400) with GPU contexts as the workers.  A call
   * carries jobs of one pubkey form (table indices or raw bytes), as the C-ABI takes one. */
  async _runJob() {
    if (this.closed) return;
    const ctx = this.ctxs.find((c) => c.inflight === 0);
    if (!ctx || this.jobs.length === 0) return;
    const isRaw = (j) => j.workReq.sets.some((s) => s.pubkey !== undefined);
    const kind = isRaw(this.jobs[0]);
    const jobs = [];
    const rest = [];
    let total = 0;
    while (this.jobs.length > 0) {
      const j = this.jobs.shift();
      if (total < this.maxSetsPerCall && isRaw(j) === kind) {
        jobs.push(j);
        total += j.workReq.sets.length;
      } else {
        rest.push(j);
        if (total >= this.maxSetsPerCall) break;
      }
    }
    this.jobs = rest.concat(this.jobs);
    const tp = this.metrics && this.metrics.blsThreadPool;
    this.stats.jobGroupsStarted += 1;
    this.stats.jobsStarted += jobs.length;
    this.stats.sigSetsStarted += total;
    if (tp) {
      for (const j of jobs) tp.jobWaitTime.observe((Date.now() - j.addedTimeMs) / 1000);
      tp.totalJobsGroupsStarted.inc(1);
      tp.totalJobsStarted.inc(jobs.length);
      tp.totalSigSetsStarted.inc(total);
    }
    if (this.jobs.length > 0) setTimeout(() => this._runJob(), 0); // another idle context may take the rest
    let verdicts;
    const t0 = process.hrtime.bigint();
    try {
      verdicts = await this._call(ctx, jobs.map((j) => j.workReq));
    } catch (e) {
      for (const j of jobs) j.reject(e);
      if (tp) tp.errorJobsSignatureSetsCount.inc(total);
      setTimeout(() => this._runJob(), 0);
      return;
    }
    if (tp) tp.jobsWorkerTime.inc({workerId: ctx.id}, Number(process.hrtime.bigint() - t0) / 1e9);
    let ok = 0;
    let err = 0;
    jobs.forEach((j, i) => {
      try {
        j.resolve(this._settle(verdicts, i));
        ok += j.workReq.sets.length;
      } catch (e) {
        j.reject(e);
        err += j.workReq.sets.length;
      }
    });
    if (tp) {
      tp.successJobsSignatureSetsCount.inc(ok);
      tp.errorJobsSignatureSetsCount.inc(err);
    }
    setTimeout(() => this._runJob(), 0);
  }
}

module.exports = {GpuBlsVerifier, chunkifyMaximizeChunkSize, packRequests, getAggregatedPubkeysCount, ERROR_MESSAGES};
