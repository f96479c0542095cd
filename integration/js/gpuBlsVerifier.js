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
 * verifyOnMainThread calls (and the synchronous state-transition helpers) run on a
 * dedicated high-priority context (bls_gpu_init_priority): the reference runs them on
 * the main thread outside the worker queue (index.ts:138-151), so they never wait
 * behind a pool call here either.  Each context runs its calls on a libuv worker
 * (napi_async_work): the process needs UV_THREADPOOL_SIZE >= contexts + 2 (pool
 * contexts, the main-thread lane, one spare), set in the environment BEFORE Node starts
 * (libuv sizes its pool once, when anything first uses it -- any fs call of a beacon
 * node does, long before this module loads -- so setting it from JS is too late).  The
 * constructor warns when the pool the process started with (UV_THREADPOOL_SIZE at
 * module load, libuv's 4 when unset) is smaller than contexts + 2.
 *
 * Contexts: the library admits a context only while the HIP runtime's scratch for the
 * process's contexts fits its budget (bls_gpu_init_priority, BLS_ERR_ADMISSION).  As the
 * reference's pool keeps the workers that started and records the others
 * (multithread/index.ts:221-229), a refused or failed pool context is recorded in
 * `initErrors` and the pool runs on the rest; when none started, queued work rejects
 * with the first error (index.ts:247-253).  The main-thread lane is opened first.
 *
 * A signature set is {pubkeyIndices: number[]} (indices into the device pubkey
 * table loaded with loadPubkeys, i.e. index2pubkey) or {pubkey: Uint8Array(96)}
 * (uncompressed affine, the worker wire format of index.ts:126), plus
 * {signingRoot: Uint8Array(32), signature: Uint8Array}.
 * Plain CommonJS so it runs on the Node in this image (v12); the TypeScript
 * version is the same code with the reference's types.
 */
const path = require("path");

const ADDON_PATH = path.join(__dirname, "..", "..", "lodestar_amd", "_native", "lodestar_bls.node");
let defaultAddon = null;
const DEFAULT_HW_QUEUES = 24;

/** The addon, loaded once.  HIP reads GPU_MAX_HW_QUEUES once, when the runtime
 * initialises, and its default of 4 queues makes more than 4 contexts serialise (12 x 22
 * calls: 2.27M sets/s on 4 queues, 3.65M on 24); the library never writes the
 * environment itself (include/lodestar_bls.h bls_gpu_request_hw_queues), so the host
 * does, here, before the addon's first HIP call -- unless the variable is set already or
 * BLS_KEEP_HW_QUEUES=1.  (A process whose HIP came up earlier keeps its count; the
 * library then warns once on stderr.) */
function loadAddon() {
  if (defaultAddon === null) {
    if (!process.env.GPU_MAX_HW_QUEUES && !process.env.BLS_KEEP_HW_QUEUES) {
      process.env.GPU_MAX_HW_QUEUES = String(DEFAULT_HW_QUEUES);
    }
    defaultAddon = require(ADDON_PATH);
  }
  return defaultAddon;
}
// the libuv pool this process started with (see the header comment): read, never written
const UV_POOL_AT_LOAD = Number(process.env.UV_THREADPOOL_SIZE || 4);
let warnedPoolSize = false;

const MAX_SIGNATURE_SETS_PER_JOB = 128; // multithread/index.ts:39
const GPU_SETS_PER_CALL = 1024; // sets per bls_gpu_verify call (cfg2 shape)
const MAX_BUFFERED_SIGS = 32; // multithread/index.ts:48
const MAX_BUFFER_WAIT_MS = 100; // multithread/index.ts:57
const SPLIT_CALL_MIN_SETS = 4096; // non-batchable calls this large are split across device slots
const AGG_KEY_WEIGHT = 1024; // keys of an aggregate set per set of routing weight (setWeight)

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

/** Pack BlsWorkReq-like jobs ({batchable, sets}) into the SoA request of bls_gpu_verify.
 * One pass to size the buffers, one to fill them; the buffers are allocated unfilled
 * (every byte the library reads is written: bytes past a short signature's length are
 * ignored, include/lodestar_bls.h). */
function packRequests(jobs, seed) {
  const nReq = jobs.length;
  let nSets = 0;
  let nIdx = 0;
  let raw = false;
  for (let r = 0; r < nReq; r++) {
    const ss = jobs[r].sets;
    nSets += ss.length;
    for (let i = 0; i < ss.length; i++) {
      const s = ss[i];
      if (s.pubkey !== undefined) raw = true;
      else nIdx += s.pubkeyIndices.length;
    }
  }
  const reqSetOffsets = new Uint32Array(nReq + 1);
  const reqBatchable = new Uint8Array(Math.max(nReq, 1));
  const messages = Buffer.allocUnsafe(Math.max(32 * nSets, 1));
  const signatures = Buffer.allocUnsafe(Math.max(96 * nSets, 1));
  let lens = null;
  const pubkeys = raw ? Buffer.allocUnsafe(96 * nSets) : null;
  const setPkOffsets = raw ? null : new Uint32Array(nSets + 1);
  const pkIndices = raw ? null : new Uint32Array(Math.max(nIdx, 1));
  let k = 0;
  let q = 0;
  for (let r = 0; r < nReq; r++) {
    const j = jobs[r];
    reqBatchable[r] = j.batchable ? 1 : 0;
    const ss = j.sets;
    for (let i = 0; i < ss.length; i++) {
      const s = ss[i];
      const root = s.signingRoot;
      if (root.length !== 32) throw Error("signing roots are 32 bytes");
      messages.set(root, 32 * k);
      const sig = s.signature;
      if (sig.length === 96) {
        signatures.set(sig, 96 * k);
      } else {
        if (lens === null) lens = new Uint32Array(nSets).fill(96);
        lens[k] = sig.length;
        signatures.set(sig.length > 96 ? sig.subarray(0, 96) : sig, 96 * k);
      }
      if (raw) {
        if (s.pubkey === undefined) throw Error("mixed raw / table pubkeys in one call");
        if (s.pubkey.length !== 96) throw Error("raw pubkeys are 96 bytes (uncompressed affine)");
        pubkeys.set(s.pubkey, 96 * k);
      } else {
        const ix = s.pubkeyIndices;
        for (let t = 0; t < ix.length; t++) pkIndices[q++] = ix[t];
        setPkOffsets[k + 1] = q;
      }
      k++;
    }
    reqSetOffsets[r + 1] = k;
  }
  return {reqSetOffsets, reqBatchable, messages, signatures, signatureLens: lens, pubkeys, setPkOffsets, pkIndices,
          seed: seed || null};
}

/** Contiguous [beg, end) shards of n sets over `parts` devices, sizes differing by at
 * most one (lodestar_amd/shard.py shard_bounds): set i keeps its call index, so its
 * random scalar is the same whichever device holds it. */
function shardBounds(n, parts) {
  const q = Math.floor(n / parts);
  const r = n % parts;
  const out = [];
  let beg = 0;
  for (let k = 0; k < parts; k++) {
    const end = beg + q + (k < r ? 1 : 0);
    out.push([beg, end]);
    beg = end;
  }
  return out;
}

/** Routing weight of a set: 1, or 1 + k / 1024 for an aggregate of k table keys (a G1
 * addition is ~11 of a set's ~12.7k Fp products; lodestar_amd/verifier.py set_weight). */
function setWeight(s) {
  const ix = s.pubkeyIndices;
  return ix !== undefined && ix.length > 1 ? 1 + ix.length / AGG_KEY_WEIGHT : 1;
}

/** SSZ kinds of bls_gpu_ssz_roots (include/lodestar_bls.h; low 8 bits = serialized size) */
const SSZ_KINDS = {
  root: 0x000 | 32,
  uint64: 0x100 | 8,
  checkpoint: 0x200 | 40,
  attestationData: 0x300 | 128,
  voluntaryExit: 0x400 | 16,
  syncAggregatorSelectionData: 0x400 | 16,
  beaconBlockHeader: 0x500 | 112,
  depositMessage: 0x600 | 88,
  forkData: 0x700 | 36,
  signingData: 0x800 | 64,
};

/** getAggregatedPubkeysCount (chain/bls/utils.ts:18-26): keys of aggregate-type sets */
function getAggregatedPubkeysCount(sets) {
  let n = 0;
  for (const s of sets) {
    const agg = s.type !== undefined ? s.type === "aggregate" : s.pubkeyIndices !== undefined && s.pubkeyIndices.length > 1;
    if (agg && s.pubkeyIndices !== undefined) n += s.pubkeyIndices.length;
  }
  return n;
}

/** A queued job: its BlsWorkReq ({batchable, sets}) and its promise's handlers. */
class Job {
  constructor(resolve, reject, batchable, sets, addedTimeMs) {
    this.resolve = resolve;
    this.reject = reject;
    this.batchable = batchable;
    this.sets = sets;
    this.addedTimeMs = addedTimeMs;
  }
}

// one executor for every job promise (no closure per job): it hands the handlers over
let capturedResolve = null;
let capturedReject = null;
function captureHandlers(resolve, reject) {
  capturedResolve = resolve;
  capturedReject = reject;
}

const NO_OPTS = {};

class GpuBlsVerifier {
  constructor(opts = {}) {
    // device slots: `devices` (one verifier per node: every GPU of the process, or a GPU
    // twice for a test of the routing on one card), else the one `device`
    const devices = Array.isArray(opts.devices) && opts.devices.length > 0 ? opts.devices.slice() : [opts.device || 0];
    const contexts = opts.contexts || 2;
    this.devices = devices;
    this.blsVerifyAllMultiThread = Boolean(opts.blsVerifyAllMultiThread);
    this.maxSetsPerCall = opts.maxSetsPerCall || GPU_SETS_PER_CALL;
    this.splitCallMinSets = Math.max(2, opts.splitCallMinSets || SPLIT_CALL_MIN_SETS);
    this.metrics = opts.metrics || null; // {bls: {...}, blsThreadPool: {...}} with the reference's names
    // the N-API addon (opts.addon: a stand-in with the same functions, for host-side tests)
    this.addon = opts.addon || loadAddon();
    const addon = this.addon;
    // the main-thread lane first: its own high-priority context on the first device,
    // never used by the pool
    this.mainCtx = {handle: addon.init(devices[0], true), inflight: 0, id: "main", slot: 0};
    this.ctxs = [];
    this.initErrors = [];
    this.nSlots = devices.length;
    this.slotCtxs = [];
    // `inflight`: calls queued or running on the context (at most one pool call each)
    for (let slot = 0; slot < devices.length; slot++) {
      const mine = [];
      for (let i = 0; i < contexts; i++) {
        try {
          const c = {handle: addon.init(devices[slot], false), inflight: 0, id: this.ctxs.length, slot};
          this.ctxs.push(c);
          mine.push(c);
        } catch (e) {
          this.initErrors.push(e); // a worker that failed to start (index.ts:221-229)
        }
      }
      this.slotCtxs.push(mine);
    }
    const uvSize = opts.uvThreadpoolSize || UV_POOL_AT_LOAD;
    const warn = opts.warn || ((m) => console.warn(m));
    if (this.ctxs.length + 2 > uvSize && (opts.warn || !warnedPoolSize)) {
      warnedPoolSize = true;
      warn(`GpuBlsVerifier: the libuv pool has ${uvSize} threads < contexts + 2 = ${this.ctxs.length + 2}; ` +
        "GPU calls will queue for libuv threads (set UV_THREADPOOL_SIZE in the environment before starting node)");
    }
    this.jobs = []; // queue: jobs[jobsHead..] are pending
    this.jobsHead = 0;
    this.runScheduled = false;
    this.bufJobs = []; // batchable jobs waiting for > 32 sigs or 100 ms (index.ts:262-279)
    this.bufSigs = 0;
    this.bufFirstMs = 0;
    this.bufTimer = null;
    this.slotLoad = new Array(this.nSlots).fill(0); // set weight each slot is running
    this.pinned = []; // per slot: shards of split calls (bls_gpu_partial)
    for (let k = 0; k < this.nSlots; k++) this.pinned.push([]);
    this.closed = false;
    this.stats = {jobsStarted: 0, sigSetsStarted: 0, jobGroupsStarted: 0, batchRetries: 0, batchSigsSuccess: 0};
    this.slotStats = this.slotCtxs.map(() => ({calls: 0, sets: 0, weight: 0}));
    this.splitStats = {calls: 0, rerouted: 0, failed: 0, badShards: []};
    this._onBufTimer = this._onBufTimer.bind(this);
    this._dispatch = this._dispatch.bind(this);
    const tp = this.metrics && this.metrics.blsThreadPool;
    // queueLength: sampled on collect, as index.ts:130 does
    if (tp && tp.queueLength && typeof tp.queueLength.addCollect === "function") {
      tp.queueLength.addCollect(() => tp.queueLength.set(this.queueLength()));
    }
  }

  /** Jobs waiting for a context (blsThreadPool.queueLength, index.ts:130) */
  queueLength() {
    return this.jobs.length - this.jobsHead;
  }

  /** Append validator pubkeys (48 B compressed each) to every context's device table on
   * every device.  All or nothing (bls_gpu_load_pubkeys appends no key of a batch holding
   * a bad one), so indices stay aligned across contexts and devices. */
  loadPubkeys(pks48) {
    [this.mainCtx].concat(this.ctxs).forEach((c, i) => {
      const codes = this.addon.loadPubkeys(c.handle, pks48, 48);
      const bad = codes.findIndex((x) => x !== 0);
      if (bad >= 0) throw Error(i === 0 ? `invalid pubkey at batch index ${bad}; no key appended` : "pubkey tables diverged");
    });
  }

  /** IBlsVerifier.verifySignatureSets (index.ts:134-174).  Returns a Promise<boolean>. */
  verifySignatureSets(sets, opts) {
    const o = opts || NO_OPTS;
    if (this.metrics) this.metrics.bls.aggregatedPubkeys.inc(getAggregatedPubkeysCount(sets));
    if (o.verifyOnMainThread && !this.blsVerifyAllMultiThread) {
      // "don't buffer": one non-batchable request now (verifySignatureSetsMaybeBatch)
      const timer = this.metrics && this.metrics.blsThreadPool.mainThreadDurationInThreadPool.startTimer();
      return this._call(this.mainCtx, [{batchable: false, sets}]).then(
        (v) => {
          if (timer) timer();
          return this._settle(v, 0);
        },
        (e) => {
          if (timer) timer();
          throw e;
        }
      );
    }
    const n = sets.length;
    const batchable = o.batchable === true;
    // one job (chunkifyMaximizeChunkSize gives one chunk): the job resolves to the
    // boolean verdict, so it is the call's result
    if (n > 0 && n <= MAX_SIGNATURE_SETS_PER_JOB) return this._queue(batchable, sets);
    if (!batchable && n >= this.splitCallMinSets && this.nSlots > 1 && this.slotCtxs.every((c) => c.length > 0)) {
      return this._splitCall(sets);
    }
    return this._queueCall(sets, batchable);
  }

  /** The reference's path for a call: chunkifyMaximizeChunkSize(sets, 128) jobs, AND-ed. */
  _queueCall(sets, batchable) {
    return Promise.all(
      chunkifyMaximizeChunkSize(sets, MAX_SIGNATURE_SETS_PER_JOB).map((chunk) => this._queue(batchable, chunk))
    ).then((results) => {
      if (results.length === 0) throw Error("Empty results array");
      return results.every((v) => v === true);
    });
  }

  /**
   * A non-batchable call of >= splitCallMinSets sets split over the device slots: each
   * slot computes the Fp12 Miller-loop partial of a contiguous shard (addon.partial =
   * bls_gpu_partial, random scalars from the call's shared seed at each set's call
   * index, so the shards form ONE random-scalar batch), the partials are gathered here
   * and one final exponentiation decides (addon.finalCheck).  The verdict equals the
   * reference's AND over the call's 128-set jobs (index.ts:153-173; each job one batch,
   * maybeBatch.ts:16-39); a failing call is localised to its shards (splitStats). When a
   * shard holds a set that does not decode, the call re-runs as the reference's jobs, so
   * the rejection is the one its Promise.all gives.
   */
  _splitCall(sets) {
    if (this.closed) return Promise.reject(Error("QUEUE_ABORTED"));
    const seed = require("crypto").randomBytes(32);
    const bounds = shardBounds(sets.length, this.nSlots);
    return new Promise((resolve, reject) => {
      const results = new Array(bounds.length);
      let pending = bounds.length;
      const done = (k, r, ctx) => {
        results[k] = r;
        if (--pending === 0) this._finishSplit(sets, results, ctx).then(resolve, reject);
      };
      bounds.forEach(([b, e], k) =>
        this.pinned[k].push({sets: sets.slice(b, e), base: b, seed, done: (r, ctx) => done(k, r, ctx)}));
      this._scheduleRun();
    });
  }

  async _finishSplit(sets, results, ctx) {
    const err = results.find((r) => r instanceof Error);
    if (err) throw err;
    if (results.some((r) => r.status !== 0)) {
      this.splitStats.rerouted++;
      return this._queueCall(sets, false);
    }
    const all = new Uint8Array(576 * results.length);
    results.forEach((r, k) => all.set(r.partial, 576 * k));
    const ok = await this._run(ctx, () => this.addon.finalCheck(ctx.handle, all));
    this.splitStats.calls++;
    if (!ok) {
      this.splitStats.failed++;
      const bad = [];
      for (let k = 0; k < results.length; k++) {
        if (!(await this._run(ctx, () => this.addon.finalCheck(ctx.handle, results[k].partial)))) bad.push(k);
      }
      this.splitStats.badShards = bad;
    }
    const tp = this.metrics && this.metrics.blsThreadPool;
    if (tp) tp.successJobsSignatureSetsCount.inc(sets.length);
    return ok;
  }

  /**
   * state-transition verifySignatureSet (src/util/signatureSets.ts:24-38) on the GPU,
   * synchronous like the reference (which blocks the main thread in blst): one
   * non-batchable request of one set (single, or aggregate with pubkeyIndices of length
   * > 1 = verifyAggregate), true / false, throwing the blst-style error when the
   * signature does not decode (Signature.fromBytes(sig, undefined, true)).
   */
  verifySignatureSetSync(set) {
    return this._settle(this.addon.verifySync(this.mainCtx.handle, packRequests([{batchable: false, sets: [set]}])), 0);
  }

  /** verifySignatureSet over many sets in one GPU call (e.g. every inline check of a
   * block when batch verification is off): per set {valid: boolean, error?: Error} --
   * valid is false with the Error its own verifySignatureSet would throw when the
   * signature does not decode, so a truthiness check of `valid` can never pass it; one
   * bad set does not hide the other sets' verdicts (lodestar_amd/stf.py likewise). */
  verifySignatureSetsEachSync(sets) {
    const v = this.addon.verifySync(this.mainCtx.handle, packRequests(sets.map((s) => ({batchable: false, sets: [s]}))));
    return sets.map((_, i) => {
      try {
        return {valid: this._settle(v, i)};
      } catch (e) {
        return {valid: false, error: e};
      }
    });
  }

  /**
   * computeSigningRoot (state-transition/src/util/signingRoot.ts:7-13) for a batch of
   * serialized SSZ objects of one kind on the GPU (SSZ_KINDS: attestationData,
   * beaconBlockHeader, uint64, ...): Uint8Array(32 n) of signing roots; `domains` is one
   * 32-byte domain, one per object, or null for the objects' hash_tree_roots.
   */
  computeSigningRoots(kind, objs, domains) {
    const k = typeof kind === "string" ? SSZ_KINDS[kind] : kind;
    if (k === undefined) throw Error(`unknown SSZ kind ${kind}`);
    return this.addon.sszRoots(this.mainCtx.handle, k, objs, domains === undefined ? null : domains);
  }

  /** IBlsVerifier.close (index.ts:176-197): abort queued jobs, wait for calls in flight */
  async close() {
    this.closed = true;
    if (this.bufTimer) clearTimeout(this.bufTimer);
    this.bufTimer = null;
    const pending = this.jobs.slice(this.jobsHead).concat(this.bufJobs);
    const pinned = [].concat(...this.pinned);
    this.jobs = [];
    this.jobsHead = 0;
    this.bufJobs = [];
    this.bufSigs = 0;
    this.pinned = this.pinned.map(() => []);
    for (const j of pending) j.reject(Error("QUEUE_ABORTED"));
    for (const p of pinned) p.done(Error("QUEUE_ABORTED"), null);
    const all = this.mainCtx ? this.ctxs.concat([this.mainCtx]) : this.ctxs;
    while (all.some((c) => c.inflight > 0)) await new Promise((r) => setTimeout(r, 5));
    for (const c of all) this.addon.close(c.handle);
    this.ctxs = [];
    this.slotCtxs = this.slotCtxs.map(() => []);
    this.mainCtx = null;
  }

  _settle(verdicts, i) {
    const code = verdicts[i];
    if (code < 0) throw Error(ERROR_MESSAGES[-code] || `BLST_ERROR: ${-code}`);
    return code === 1;
  }

  async _call(ctx, jobs) {
    if (this.closed && this.ctxs.length === 0) throw Error("QUEUE_ABORTED");
    return this._run(ctx, () => this.addon.verify(ctx.handle, packRequests(jobs)));
  }

  /** run fn (an addon call returning a promise) with the context counted in flight */
  async _run(ctx, fn) {
    ctx.inflight++;
    try {
      return await fn();
    } finally {
      ctx.inflight--;
    }
  }

  /** queueBlsWork (index.ts:238-285) */
  _queue(batchable, sets) {
    if (this.closed) return Promise.reject(Error("QUEUE_ABORTED"));
    // every pool context failed to start: the first error (index.ts:247-253)
    if (this.ctxs.length === 0 && this.initErrors.length > 0) return Promise.reject(this.initErrors[0]);
    const promise = new Promise(captureHandlers);
    const job = new Job(capturedResolve, capturedReject, batchable, sets, this.metrics ? Date.now() : 0);
    if (batchable) {
      if (this.bufJobs.length === 0) {
        this.bufFirstMs = Date.now();
        // one timer at a time: a buffer flushed by its size leaves it armed, and when it
        // fires it re-arms for the current buffer's remaining wait
        if (this.bufTimer === null) this.bufTimer = setTimeout(this._onBufTimer, MAX_BUFFER_WAIT_MS);
      }
      this.bufJobs.push(job);
      this.bufSigs += sets.length;
      if (this.bufSigs > MAX_BUFFERED_SIGS) this._flushBuffer();
    } else {
      this.jobs.push(job);
      this._scheduleRun();
    }
    return promise;
  }

  _onBufTimer() {
    this.bufTimer = null;
    if (this.bufJobs.length === 0 || this.closed) return;
    const wait = this.bufFirstMs + MAX_BUFFER_WAIT_MS - Date.now();
    if (wait <= 0) this._flushBuffer();
    else this.bufTimer = setTimeout(this._onBufTimer, wait);
  }

  _flushBuffer() {
    const buf = this.bufJobs;
    if (this.jobsHead >= this.jobs.length) {
      this.jobs = buf; // queue empty: take the buffer's array as the queue
      this.jobsHead = 0;
    } else {
      for (let i = 0; i < buf.length; i++) this.jobs.push(buf[i]);
    }
    this.bufJobs = [];
    this.bufSigs = 0;
    this._scheduleRun();
  }

  /** setTimeout(runJob, 0) (index.ts:282,409): one pending dispatch at a time */
  _scheduleRun() {
    if (this.runScheduled) return;
    this.runScheduled = true;
    setImmediate(this._dispatch);
  }

  /** An idle context of the slot, or null */
  _idleCtx(slot) {
    const cs = this.slotCtxs[slot];
    for (let i = 0; i < cs.length; i++) if (cs[i].inflight === 0) return cs[i];
    return null;
  }

  /** runJob / prepareWork (index.ts:290-400) with GPU contexts as the workers, over every
   * device slot: split-call shards go to their own slot; queued jobs go to an idle
   * context of the slot carrying the least set weight in flight (least-loaded device). */
  _dispatch() {
    this.runScheduled = false;
    if (this.closed) return;
    for (;;) {
      for (let s = 0; s < this.nSlots; s++) {
        while (this.pinned[s].length > 0) {
          const ctx = this._idleCtx(s);
          if (ctx === null) break;
          this._startPinned(ctx, this.pinned[s].shift());
        }
      }
      if (this.jobsHead >= this.jobs.length) return;
      let ctx = null;
      let best = Infinity;
      for (let s = 0; s < this.nSlots; s++) {
        if (this.slotLoad[s] >= best) continue;
        const c = this._idleCtx(s);
        if (c !== null) {
          ctx = c;
          best = this.slotLoad[s];
        }
      }
      if (ctx === null) return;
      this._startJobs(ctx);
    }
  }

  _startPinned(ctx, p) {
    const w = p.sets.length;
    this.slotLoad[ctx.slot] += w;
    const st = this.slotStats[ctx.slot];
    st.calls++;
    st.sets += p.sets.length;
    st.weight += w;
    const tp = this.metrics && this.metrics.blsThreadPool;
    if (tp) {
      tp.totalJobsGroupsStarted.inc(1);
      tp.totalJobsStarted.inc(1);
      tp.totalSigSetsStarted.inc(p.sets.length);
    }
    let req;
    try {
      req = packRequests([{batchable: false, sets: p.sets}], p.seed);
    } catch (e) {
      this.slotLoad[ctx.slot] -= w;
      p.done(e, ctx);
      return;
    }
    this._run(ctx, () => this.addon.partial(ctx.handle, req, p.base)).then(
      (r) => {
        this.slotLoad[ctx.slot] -= w;
        p.done(r, ctx);
        this._dispatch();
      },
      (e) => {
        this.slotLoad[ctx.slot] -= w;
        p.done(e, ctx);
        this._dispatch();
      }
    );
  }

  /** Take queued jobs of one pubkey form (table indices or raw bytes) for one call and
   * start it.  A raw-key call is one worker message as prepareWork builds it (jobs until
   * >= 128 sets): a key that does not decode rejects every job of its message
   * (deserializeSet, worker.ts:43-46), so it must not take more jobs with it than the
   * reference's message would.  Table-index calls cannot fail that way and take up to
   * maxSetsPerCall sets. */
  _startJobs(ctx) {
    const q = this.jobs;
    const first = q[this.jobsHead];
    const kind = first.sets[0] !== undefined && first.sets[0].pubkey !== undefined;
    const jobs = [];
    let skipped = null;
    let total = 0;
    let weight = 0;
    const cap = kind ? MAX_SIGNATURE_SETS_PER_JOB : this.maxSetsPerCall;
    while (this.jobsHead < q.length && total < cap) {
      const j = q[this.jobsHead];
      q[this.jobsHead++] = undefined;
      const s0 = j.sets[0];
      if ((s0 !== undefined && s0.pubkey !== undefined) === kind) {
        jobs.push(j);
        const ss = j.sets;
        total += ss.length;
        for (let i = 0; i < ss.length; i++) weight += setWeight(ss[i]);
      } else {
        (skipped || (skipped = [])).push(j); // other pubkey form: a later call
      }
    }
    if (skipped !== null) {
      this.jobs = skipped.concat(q.slice(this.jobsHead));
      this.jobsHead = 0;
    } else if (this.jobsHead > 4096 && this.jobsHead * 2 > q.length) {
      this.jobs = q.slice(this.jobsHead);
      this.jobsHead = 0;
    }
    const tp = this.metrics && this.metrics.blsThreadPool;
    this.stats.jobGroupsStarted += 1;
    this.stats.jobsStarted += jobs.length;
    this.stats.sigSetsStarted += total;
    const st = this.slotStats[ctx.slot];
    st.calls++;
    st.sets += total;
    st.weight += weight;
    if (tp) {
      const now = Date.now();
      for (const j of jobs) tp.jobWaitTime.observe((now - j.addedTimeMs) / 1000);
      tp.totalJobsGroupsStarted.inc(1);
      tp.totalJobsStarted.inc(jobs.length);
      tp.totalSigSetsStarted.inc(total);
    }
    this.slotLoad[ctx.slot] += weight;
    const jobStartNs = tp ? Number(process.hrtime.bigint()) : 0;
    this._call(ctx, jobs).then(
      (verdicts) => {
        this.slotLoad[ctx.slot] -= weight;
        this._settleCall(ctx, jobs, verdicts, total, jobStartNs);
        this._dispatch();
      },
      (e) => {
        this.slotLoad[ctx.slot] -= weight;
        for (const j of jobs) j.reject(e);
        if (tp) tp.errorJobsSignatureSetsCount.inc(total);
        this._dispatch();
      }
    );
  }

  /** Settle one GPU call's jobs in one pass over its verdict array. */
  _settleCall(ctx, jobs, verdicts, total, jobStartNs) {
    const tp = this.metrics && this.metrics.blsThreadPool;
    // the worker's BlsWorkResult bookkeeping (addon: properties of the verdict array)
    const retries = verdicts.batchRetries || 0;
    const sigsOk = verdicts.batchSigsSuccess || 0;
    this.stats.batchRetries += retries;
    this.stats.batchSigsSuccess += sigsOk;
    let ok = 0;
    let err = 0;
    for (let i = 0; i < jobs.length; i++) {
      const j = jobs[i];
      const code = verdicts[i];
      if (code >= 0) {
        j.resolve(code === 1);
        ok += j.sets.length;
      } else {
        j.reject(Error(ERROR_MESSAGES[-code] || `BLST_ERROR: ${-code}`));
        err += j.sets.length;
      }
    }
    if (tp) {
      const jobEndNs = Number(process.hrtime.bigint());
      const wStart = verdicts.workerStartNs !== undefined ? verdicts.workerStartNs : jobStartNs;
      const wEnd = verdicts.workerEndNs !== undefined ? verdicts.workerEndNs : jobEndNs;
      // index.ts:357-366
      tp.jobsWorkerTime.inc({workerId: ctx.id}, (wEnd - wStart) / 1e9);
      tp.latencyToWorker.observe(Math.max(0, wStart - jobStartNs) / 1e9);
      tp.latencyFromWorker.observe(Math.max(0, jobEndNs - wEnd) / 1e9);
      tp.batchRetries.inc(retries);
      tp.batchSigsSuccess.inc(sigsOk);
      tp.successJobsSignatureSetsCount.inc(ok);
      tp.errorJobsSignatureSetsCount.inc(err);
    }
  }
}

module.exports = {
  GpuBlsVerifier,
  chunkifyMaximizeChunkSize,
  packRequests,
  shardBounds,
  setWeight,
  getAggregatedPubkeysCount,
  ERROR_MESSAGES,
  SSZ_KINDS,
};
