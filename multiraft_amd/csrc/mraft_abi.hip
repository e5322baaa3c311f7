// mraft_abi.hip — the extern "C" boundary of libmraft_hip.so (include/mraft.h).
//
// Host side of the engine: device state ownership (one HBM-resident SoA image
// per handle), staging of host batches, duplicate-slot claims and kernel
// launches on the handle's stream. No exception or C++ type crosses the ABI.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mraft.h"
#include "mraft_device.h"
#include "mraft_internal.h"

constexpr int kMaxShards = 8;
// Default capacity of the AppendEntries stage (mraft_set_stage_capacity): 16 MiB.
constexpr int64_t kDefaultStageWords = (int64_t)1 << 22;
// The deferred launch's grid (mraft_handle_append_entries by reference): the
// last call's deferred count, read from a pinned word the device writes, in
// [kDeferGridMin, kDeferGridMax] workgroups (grid-stride beyond). With no
// deferred item the launch exits at once on kDeferGridMin workgroups; a
// deferred-heavy batch gets a workgroup per item from the next call on. The
// minimum bounds the first deferred-heavy call after calls without any (a
// partition healing): 512 workgroups take it 30.6 -> 1.07 ms (stale second
// leaders) and 96.9 -> 3.7 ms (2-cycles) against 8, with the message path's
// pipelines within noise (profiles/r6_g1; round 5 had chosen 8 for ~2 %
// there, r5_g1).
#ifndef MRAFT_DEFER_GRID_MIN
#define MRAFT_DEFER_GRID_MIN 512
#endif
constexpr int kDeferGridMin = MRAFT_DEFER_GRID_MIN;
constexpr int kDeferGridMax = 1 << 16;
// The light tick's fallback launch (MRAFT_TICK_LIGHT): at least this many
// workgroups, twice the previous light tick's count, at most the groups (a
// grid-stride loop makes any grid exact; an empty one costs a few µs).
constexpr long long kLiteGridMin = 2048;
constexpr long long kLiteGridUnknown = 8192;
constexpr int kAutoProbe = 32;  // MRAFT_TICK_AUTO: a light tick at least every 32 ticks
// The engine's pinned host words (device-written, read by the host when it
// enqueues): [0] the last by-reference AppendEntries call's deferred count,
// [1] the staged words of the last call that exceeded the stage (its need),
// [kHintLite + s] the last light tick's fallback count of shard s.
constexpr int kHintLite = 2;
constexpr int kHintWords = kHintLite + kMaxShards;
// MRAFT_STAGE_AUTO grows the stage to 5/4 of a batch's need, in 1 Mi-word
// steps, up to 2^31 - 1 words (8 GiB).
constexpr int64_t kStageStep = (int64_t)1 << 20;
// Words of the fallback's per-workgroup cycle buffers (nslot x L, at most this).
constexpr int64_t kCycSlotWords = (int64_t)1 << 25;  // 8,192 buffers at L = 4,096 (128 MiB)

struct mraft_engine {
  int32_t G = 0, P = 0, L = 0, device = 0;
  bool owned = false, bound = false;
  mraft_soa dev{};
  hipStream_t own_stream = nullptr, stream = nullptr;
  // fan-in (mraft_allgather_status): its own stream, ordered after the engine
  // stream by an event; optional CU-masked pair (mraft_fanin_reserve_cus)
  hipStream_t fanin_own = nullptr, fanin_masked = nullptr, tick_masked = nullptr;
  hipEvent_t fanin_ev = nullptr;
  int32_t fan_cus = 0;  // CUs reserved for the fan-in (the tick side's masks leave them out)
  // Tick group shards (mraft_set_tick_shards): S dedicated hardware queues the
  // engine owns; a tick forks onto them from the engine stream (fork_ev) and
  // the next call of any other kind joins them back (shard_ev), so one shard's
  // tick i+1 follows only its own tick i.
  int32_t nshards = 1;
  hipStream_t shard_q[kMaxShards] = {};
  hipEvent_t shard_ev[kMaxShards] = {};
  hipEvent_t fork_ev = nullptr;
  bool shards_pending = false;
  unsigned long long *claim = nullptr;
  uint32_t *srcmark = nullptr;             // per slot: epoch of the last call that read its row
  uint32_t epoch = 0;
  unsigned long long *ae_total = nullptr;  // AppendEntries by reference: the deferred launch's counters (mraft_kernels.hip)
  int64_t stage_cap = kDefaultStageWords;  // words of staged entries the deferred launch may use
  bool stage_auto = true;                  // MRAFT_STAGE_AUTO: grow stage_cap to the last overflow's need
  long long *dhint = nullptr;  // pinned host word: the last by-reference call's deferred count (device-written)
  long long *dhint_dev = nullptr;  // its device-side address
  // the deferred launch's minimum grid: kDeferGridMin, or the environment's
  // MRAFT_DEFER_GRID_MIN at mraft_create (tests run the small-grid paths with it)
  long long defer_grid_min = kDeferGridMin;
  // MRAFT_TICK_LIGHT (mraft_set_tick_mode): the lists of groups for the full
  // tick (shard s at its first group + 512 s), a pair of counter sets per shard (the light
  // launch counts into one, the fallback zeroes the other for the next tick)
  // and per shard the last fallback count, pinned (dhint + kHintLite + s)
  int32_t tick_mode = MRAFT_TICK_AUTO;
  int32_t *lite_list = nullptr;
  unsigned *lite_cnt = nullptr;
  int lite_par[kMaxShards] = {};
  int auto_since[kMaxShards] = {};  // MRAFT_TICK_AUTO: full ticks since the last light one
  std::vector<void *> scratch_ptr;
  std::vector<size_t> scratch_cap;
};

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail(MRAFT_E_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));          \
  } while (0)

#define TRY(expr)          \
  do {                     \
    int rc_ = (expr);      \
    if (rc_) return rc_;   \
  } while (0)

int64_t gp_of(const mraft_engine *h) { return (int64_t)h->G * h->P; }

mraft::Dev dev_of(const mraft_engine *h) {
  mraft::Dev d;
  d.term = h->dev.current_term; d.voted = h->dev.voted_for; d.role = h->dev.state;
  d.commit = h->dev.commit_index; d.applied = h->dev.last_applied; d.dummy = h->dev.dummy_index;
  d.last = h->dev.last_index; d.votes = h->dev.granted_votes; d.log = h->dev.log_term;
  d.match = h->dev.match_index; d.next = h->dev.next_index; d.pdirty = h->dev.persist_dirty;
  d.head = h->dev.log_head; d.hsnap = h->dev.has_snapshot; d.srt = h->dev.terms_sorted;
  d.G = h->G; d.P = h->P; d.L = h->L;
  return d;
}

// Array table: pointer-to-member + element count.
struct ArrDesc { int32_t *mraft_soa::*ptr; int kind; };  // kind 0: G*P, 1: G*P*L, 2: G*P*P
const ArrDesc kArrays[] = {
    {&mraft_soa::current_term, 0}, {&mraft_soa::voted_for, 0},   {&mraft_soa::state, 0},
    {&mraft_soa::commit_index, 0}, {&mraft_soa::last_applied, 0}, {&mraft_soa::dummy_index, 0},
    {&mraft_soa::last_index, 0},   {&mraft_soa::granted_votes, 0}, {&mraft_soa::log_term, 1},
    {&mraft_soa::match_index, 2},  {&mraft_soa::next_index, 2},  {&mraft_soa::persist_dirty, 0},
    {&mraft_soa::log_head, 0},     {&mraft_soa::has_snapshot, 0}, {&mraft_soa::terms_sorted, 0}};

size_t arr_bytes(const mraft_engine *h, int kind) {
  int64_t gp = gp_of(h);
  int64_t n = kind == 0 ? gp : kind == 1 ? gp * h->L : gp * h->P;
  return (size_t)n * sizeof(int32_t);
}

int check(const mraft_engine *h) {
  if (!h) return fail(MRAFT_E_INVAL, "null engine handle");
  if (!h->bound) return fail(MRAFT_E_NOSTATE, "engine has no device state bound");
  return MRAFT_OK;
}

// Orders the engine stream after every shard launch still outstanding (no
// host wait): the shard queues record their join events and the engine
// stream waits on them.
int join_shards(mraft_engine *h) {
  if (!h->shards_pending) return MRAFT_OK;
  for (int s = 0; s < h->nshards; ++s) {
    HIP_TRY(hipEventRecord(h->shard_ev[s], h->shard_q[s]));
    HIP_TRY(hipStreamWaitEvent(h->stream, h->shard_ev[s], 0));
  }
  h->shards_pending = false;
  return MRAFT_OK;
}

// Every entry point but the sharded tick: the handle is usable and earlier
// sharded ticks are ordered before this call's work on the engine stream.
int enter(mraft_engine *h) {
  int rc = check(h);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(h->device));
  return join_shards(h);
}

// Host wait for everything the engine has enqueued (engine, shard and fan-in
// streams). Errors are ignored (teardown paths).
void drain(mraft_engine *h) {
  (void)hipStreamSynchronize(h->stream);
  for (int s = 0; s < h->nshards; ++s)
    if (h->shard_q[s]) (void)hipStreamSynchronize(h->shard_q[s]);
  h->shards_pending = false;
}

// A stream on a hardware queue of its own (hipExtStreamCreateWithCUMask: a
// CU-masked stream gets a dedicated queue, a pooled stream may share one with
// another stream, and two launches on one queue run one after the other).
// tick_side: every CU but the fan-in's reserved ones; otherwise only those.
int make_queue(mraft_engine *h, bool tick_side, hipStream_t *out) {
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, h->device));
  const int ncu = prop.multiProcessorCount, nw = (ncu + 31) / 32;
  std::vector<uint32_t> mask(nw, 0);
  // the highest fan_cus CU bits go to the fan-in, the rest to the tick
  for (int cu = 0; cu < ncu; ++cu)
    if ((cu >= ncu - h->fan_cus) != tick_side) mask[cu / 32] |= 1u << (cu % 32);
  HIP_TRY(hipExtStreamCreateWithCUMask(out, (uint32_t)nw, mask.data()));
  return MRAFT_OK;
}

void destroy_shard_queues(mraft_engine *h) {
  for (int s = 0; s < kMaxShards; ++s) {
    if (h->shard_q[s]) {
      (void)hipStreamSynchronize(h->shard_q[s]);
      (void)hipStreamDestroy(h->shard_q[s]);
      h->shard_q[s] = nullptr;
    }
    if (h->shard_ev[s]) (void)hipEventDestroy(h->shard_ev[s]);
    h->shard_ev[s] = nullptr;
  }
  h->shards_pending = false;
}

int create_shard_queues(mraft_engine *h, int n) {
  for (int s = 0; s < n; ++s) {
    TRY(make_queue(h, true, &h->shard_q[s]));
    HIP_TRY(hipEventCreateWithFlags(&h->shard_ev[s], hipEventDisableTiming));
  }
  if (!h->fork_ev) HIP_TRY(hipEventCreateWithFlags(&h->fork_ev, hipEventDisableTiming));
  return MRAFT_OK;
}

// Groups [g0, g1) of the engine's state as a state of their own (the SoA
// arrays are group-major: no copies).
mraft::Dev dev_slice(const mraft_engine *h, int32_t g0, int32_t g1) {
  mraft::Dev d = dev_of(h);
  const int64_t s0 = (int64_t)g0 * h->P;
  for (int32_t **p : {&d.term, &d.voted, &d.role, &d.commit, &d.applied, &d.dummy, &d.last, &d.votes, &d.pdirty,
                      &d.head, &d.hsnap, &d.srt})
    if (*p) *p += s0;
  d.log += s0 * h->L;
  d.match += s0 * h->P;
  d.next += s0 * h->P;
  d.G = g1 - g0;
  return d;
}

int32_t *off(int32_t *p, int64_t k) { return p ? p + k : nullptr; }

// The tick launch(es): one launch on the engine stream, or with S tick shards
// one launch per contiguous group range on its own queue, each queue first
// waiting for the engine stream's prior work (one event, fork_ev).
int alloc_async(mraft_engine *h, void **p, size_t bytes, const char *what);

// The light tick's buffers (MRAFT_TICK_LIGHT), allocated on first use,
// stream-ordered, counters zeroed.
int ensure_lite(mraft_engine *h) {
  if (h->lite_list) return MRAFT_OK;
  void *l = nullptr, *c = nullptr;
  // a shard of G_s groups needs lite_list_words(G_s) <= G_s + 512 words
  TRY(alloc_async(h, &l, ((size_t)h->G + 512 * kMaxShards) * sizeof(int32_t), "light tick list"));
  h->lite_list = (int32_t *)l;
  const size_t cb = (size_t)2 * kMaxShards * mraft::kLiteCntWords * sizeof(unsigned);
  TRY(alloc_async(h, &c, cb, "light tick counters"));
  h->lite_cnt = (unsigned *)c;
  HIP_TRY(hipMemsetAsync(h->lite_cnt, 0, cb, h->stream));
  for (int s = 0; s < kMaxShards; ++s) h->lite_par[s] = 0;
  return MRAFT_OK;
}

// One tick launch over groups [g0, g0 + d.G) as shard s on stream st: the full
// tick, or the light tick's pair of launches.
// MRAFT_TICK_AUTO's choice for shard s of G_s groups: the light tick while
// the last completed light tick sent at most a quarter of the groups to the
// full tick (or none has completed yet); otherwise the full tick, with a
// light tick every kAutoProbe-th tick to measure again.
bool auto_light(mraft_engine *h, int s, int32_t gs) {
  const long long last = ((volatile long long *)h->dhint)[kHintLite + s];
  if (last < 0 || 4 * last <= (long long)gs) {
    h->auto_since[s] = 0;
    return true;
  }
  if (++h->auto_since[s] >= kAutoProbe) {
    h->auto_since[s] = 0;
    return true;
  }
  return false;
}

// sio (mraft_start_and_tick): Start at the range's leaders first — inside the
// light launch, or as its own launch before the full tick.
void tick_range(mraft_engine *h, const mraft::Dev &d, int s, int32_t g0, const int32_t *lp, int32_t *gf,
                int32_t *ec, int32_t *et, hipStream_t st, const mraft::StartIO *sio = nullptr) {
  const bool light = h->P >= 2 && (h->tick_mode == MRAFT_TICK_LIGHT ||
                                   (h->tick_mode == MRAFT_TICK_AUTO && auto_light(h, s, d.G)));
  mraft::StartIO so{};
  if (sio) so = {sio->counts + g0, sio->oi + g0, sio->ot + g0, sio->ol + g0, sio->err + g0};
  if (!light) {
    if (sio) mraft::launch_start_groups(d, lp + g0, so, st);
    mraft::launch_replicate_tick(d, lp + g0, off(gf, g0), off(ec, g0), off(et, g0), st);
    return;
  }
  mraft::LiteBufs lb;
  const int par = h->lite_par[s];
  h->lite_par[s] ^= 1;
  lb.list = h->lite_list + g0 + 512 * s;
  lb.cnt = h->lite_cnt + (2 * s + par) * mraft::kLiteCntWords;
  lb.cnt_next = h->lite_cnt + (2 * s + (par ^ 1)) * mraft::kLiteCntWords;
  lb.hint = h->dhint_dev + kHintLite + s;
  const long long prev = ((volatile long long *)h->dhint)[kHintLite + s];
  // no completed light tick yet (e.g. the first ticks enqueued back to back):
  // one wave per SIMD slot, grid-stride
  const long long gr = prev < 0 ? kLiteGridUnknown : std::max(kLiteGridMin, 2 * prev);
  lb.grid = (int)std::max(1ll, std::min(gr, (long long)d.G));
  mraft::launch_replicate_tick_light(d, lp + g0, off(gf, g0), off(ec, g0), off(et, g0), lb, sio ? &so : nullptr, st);
}

int launch_tick(mraft_engine *h, const int32_t *lp, int32_t *gf, int32_t *ec, int32_t *et,
                const mraft::StartIO *sio = nullptr) {
  if (h->tick_mode != MRAFT_TICK_FULL) TRY(ensure_lite(h));
  if (h->nshards <= 1) {
    tick_range(h, dev_of(h), 0, 0, lp, gf, ec, et, h->stream, sio);
    HIP_TRY(hipGetLastError());
    return MRAFT_OK;
  }
  HIP_TRY(hipEventRecord(h->fork_ev, h->stream));
  for (int s = 0; s < h->nshards; ++s) HIP_TRY(hipStreamWaitEvent(h->shard_q[s], h->fork_ev, 0));
  for (int s = 0; s < h->nshards; ++s) {
    const int32_t g0 = (int32_t)((int64_t)h->G * s / h->nshards), g1 = (int32_t)((int64_t)h->G * (s + 1) / h->nshards);
    if (g1 <= g0) continue;
    tick_range(h, dev_slice(h, g0, g1), s, g0, lp, gf, ec, et, h->shard_q[s], sio);
  }
  h->shards_pending = true;
  HIP_TRY(hipGetLastError());
  return MRAFT_OK;
}

// Device memory in stream order on the engine stream (hipMallocAsync /
// hipFreeAsync): allocating or growing a buffer never waits for the device, so
// MRAFT_DEVICE calls stay asynchronous when a batch is larger than any before
// (include/mraft.h). A freed buffer is released after the
// work already enqueued on the stream, which may still read it.
int alloc_async(mraft_engine *h, void **p, size_t bytes, const char *what) {
  *p = nullptr;
  if (hipMallocAsync(p, bytes, h->stream) != hipSuccess || !*p) {
    (void)hipGetLastError();
    return fail(MRAFT_E_NOMEM, "%s: device allocation of %zu B failed", what, bytes);
  }
  return MRAFT_OK;
}

// Grow-only device scratch slot `idx` (stream-ordered: no host wait).
int scratch(mraft_engine *h, size_t idx, size_t bytes, void **out) {
  if (h->scratch_ptr.size() <= idx) {
    h->scratch_ptr.resize(idx + 1, nullptr);
    h->scratch_cap.resize(idx + 1, 0);
  }
  if (bytes == 0) bytes = 16;
  if (h->scratch_cap[idx] < bytes) {
    if (h->scratch_ptr[idx]) HIP_TRY(hipFreeAsync(h->scratch_ptr[idx], h->stream));
    h->scratch_ptr[idx] = nullptr;
    h->scratch_cap[idx] = 0;
    void *p = nullptr;
    TRY(alloc_async(h, &p, bytes, "scratch"));
    h->scratch_ptr[idx] = p;
    h->scratch_cap[idx] = bytes;
  }
  *out = h->scratch_ptr[idx];
  return MRAFT_OK;
}

// scratch() whose new buffer is zeroed when it is (re)allocated (stream-ordered):
// for epoch-tagged counters, whose stale contents must never carry a tag a
// later call could take for its own.
int scratch_zeroed(mraft_engine *h, size_t idx, size_t bytes, void **out) {
  const bool grows = h->scratch_ptr.size() <= idx || h->scratch_cap[idx] < (bytes ? bytes : 16);
  TRY(scratch(h, idx, bytes, out));
  if (grows) HIP_TRY(hipMemsetAsync(*out, 0, h->scratch_cap[idx], h->stream));
  return MRAFT_OK;
}

// Batch pointer staging: for MRAFT_HOST, input buffers are copied to device
// scratch and output buffers are copied back by finish().
struct Stage {
  mraft_engine *h;
  bool host;
  size_t next_slot = 0;
  struct Out { void *host; void *dev; size_t bytes; };
  std::vector<Out> outs;
  Stage(mraft_engine *hh, int32_t where) : h(hh), host(where == MRAFT_HOST) {}

  // in: read by the kernel; out: written by the kernel; both: read and written.
  int map(const void *p, size_t bytes, bool in, bool out, void **dptr) {
    if (!p) { *dptr = nullptr; return MRAFT_OK; }
    if (!host) { *dptr = const_cast<void *>(p); return MRAFT_OK; }
    void *d = nullptr;
    int rc = scratch(h, 8 + next_slot++, bytes, &d);
    if (rc) return rc;
    if (in && bytes) HIP_TRY(hipMemcpyAsync(d, p, bytes, hipMemcpyHostToDevice, h->stream));
    if (out) outs.push_back({const_cast<void *>(p), d, bytes});
    *dptr = d;
    return MRAFT_OK;
  }
  int finish() {
    HIP_TRY(hipGetLastError());
    if (!host) return MRAFT_OK;
    for (auto &o : outs)
      if (o.bytes) HIP_TRY(hipMemcpyAsync(o.host, o.dev, o.bytes, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return MRAFT_OK;
  }
};


int ensure_claim(mraft_engine *h) {
  if (!h->claim) {
    size_t b = (size_t)gp_of(h) * sizeof(unsigned long long);
    void *c = nullptr, *m = nullptr;
    TRY(alloc_async(h, &c, b, "claim"));
    h->claim = (unsigned long long *)c;
    HIP_TRY(hipMemsetAsync(h->claim, 0, b, h->stream));
    TRY(alloc_async(h, &m, (size_t)gp_of(h) * sizeof(uint32_t), "srcmark"));
    h->srcmark = (uint32_t *)m;
    HIP_TRY(hipMemsetAsync(h->srcmark, 0, (size_t)gp_of(h) * sizeof(uint32_t), h->stream));
  }
  if (++h->epoch == 0) {  // wrapped: reset (and every epoch-tagged counter)
    HIP_TRY(hipMemsetAsync(h->claim, 0, (size_t)gp_of(h) * sizeof(unsigned long long), h->stream));
    HIP_TRY(hipMemsetAsync(h->srcmark, 0, (size_t)gp_of(h) * sizeof(uint32_t), h->stream));
    if (h->scratch_ptr.size() > 20 && h->scratch_ptr[20])
      HIP_TRY(hipMemsetAsync(h->scratch_ptr[20], 0, h->scratch_cap[20], h->stream));
    h->epoch = 1;
  }
  return MRAFT_OK;
}

void free_owned(mraft_engine *h) {
  if (!h->owned) return;
  for (const auto &a : kArrays) {
    int32_t *p = h->dev.*(a.ptr);
    if (p) (void)hipFree(p);
    h->dev.*(a.ptr) = nullptr;
  }
  h->owned = false;
  h->bound = false;
}

}  // namespace

extern "C" {

const char *mraft_last_error_string(void) { return g_err.c_str(); }
int mraft_abi_version(void) { return MRAFT_ABI_VERSION; }

int mraft_create(int32_t groups, int32_t peers, int32_t log_capacity, int32_t device,
                 uint32_t flags, mraft_engine **out) {
  if (!out) return fail(MRAFT_E_INVAL, "out is null");
  *out = nullptr;
  if (groups < 1 || peers < 1 || peers > 8 || log_capacity < 1 || log_capacity > MRAFT_MAX_LOG_CAPACITY)
    return fail(MRAFT_E_INVAL, "bad dims G=%d P=%d L=%d (need G>=1, 1<=P<=8, 1<=L<=%d)", groups, peers,
                log_capacity, MRAFT_MAX_LOG_CAPACITY);
  if ((int64_t)groups * peers > INT32_MAX)
    return fail(MRAFT_E_INVAL, "G*P must fit in int32");
  HIP_TRY(hipSetDevice(device));
  mraft_engine *h = new mraft_engine();
  h->G = groups; h->P = peers; h->L = log_capacity; h->device = device;
  if (const char *e = getenv("MRAFT_DEFER_GRID_MIN")) {
    const long long v = atoll(e);
    if (v >= 1 && v <= kDeferGridMax) h->defer_grid_min = v;
  }
  if (flags & MRAFT_CREATE_DEDICATED_QUEUE) {
    const int rc = make_queue(h, true, &h->own_stream);
    if (rc) {
      delete h;
      return rc;
    }
  } else if (hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return fail(MRAFT_E_HIP, "hipStreamCreate failed");
  }
  h->stream = h->own_stream;
  {
    void *hp = nullptr;
    if (hipHostMalloc(&hp, sizeof(long long) * kHintWords, hipHostMallocMapped) != hipSuccess) {
      (void)hipStreamDestroy(h->own_stream);
      delete h;
      return fail(MRAFT_E_NOMEM, "pinned host word allocation failed");
    }
    h->dhint = (long long *)hp;
    *(volatile long long *)h->dhint = 0;
    ((volatile long long *)h->dhint)[1] = 0;
    for (int k = 0; k < kMaxShards; ++k) ((volatile long long *)h->dhint)[kHintLite + k] = -1;  // no light tick yet
    void *dp = nullptr;
    if (hipHostGetDevicePointer(&dp, hp, 0) != hipSuccess) {
      (void)hipHostFree(hp);
      (void)hipStreamDestroy(h->own_stream);
      delete h;
      return fail(MRAFT_E_HIP, "hipHostGetDevicePointer failed");
    }
    h->dhint_dev = (long long *)dp;
  }
  if (!(flags & MRAFT_CREATE_NO_ALLOC)) {
    h->owned = true;
    for (const auto &a : kArrays) {
      int32_t *p = nullptr;
      if (hipMalloc(&p, arr_bytes(h, a.kind)) != hipSuccess) {
        free_owned(h);
        (void)hipStreamDestroy(h->own_stream);
        (void)hipHostFree(h->dhint);
        delete h;
        return fail(MRAFT_E_NOMEM, "device state allocation failed (G=%d P=%d L=%d)", groups, peers,
                    log_capacity);
      }
      h->dev.*(a.ptr) = p;
    }
    h->bound = true;
    (void)hipMemsetAsync(h->dev.log_term, 0, arr_bytes(h, 1), h->stream);
    (void)hipMemsetAsync(h->dev.match_index, 0, arr_bytes(h, 2), h->stream);
    (void)hipMemsetAsync(h->dev.next_index, 0, arr_bytes(h, 2), h->stream);
    mraft::launch_init_state(dev_of(h), h->stream);
    hipError_t e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) {
      free_owned(h);
      (void)hipStreamDestroy(h->own_stream);
      (void)hipHostFree(h->dhint);
      delete h;
      return fail(MRAFT_E_HIP, "init failed: %s", hipGetErrorString(e));
    }
  }
  *out = h;
  return MRAFT_OK;
}

int mraft_destroy(mraft_engine *h) {
  if (!h) return MRAFT_OK;
  (void)hipSetDevice(h->device);
  drain(h);
  free_owned(h);
  // stream-ordered buffers (alloc_async): freed on the engine stream, then waited for
  for (void *p : h->scratch_ptr)
    if (p) (void)hipFreeAsync(p, h->stream);
  for (void *p : {(void *)h->claim, (void *)h->srcmark, (void *)h->ae_total, (void *)h->lite_list, (void *)h->lite_cnt})
    if (p) (void)hipFreeAsync(p, h->stream);
  (void)hipStreamSynchronize(h->stream);
  if (h->fanin_own) (void)hipStreamSynchronize(h->fanin_own);
  if (h->fanin_masked) (void)hipStreamSynchronize(h->fanin_masked);
  destroy_shard_queues(h);
  for (hipStream_t s : {h->own_stream, h->fanin_own, h->fanin_masked, h->tick_masked})
    if (s) (void)hipStreamDestroy(s);
  if (h->fanin_ev) (void)hipEventDestroy(h->fanin_ev);
  if (h->fork_ev) (void)hipEventDestroy(h->fork_ev);
  if (h->dhint) (void)hipHostFree(h->dhint);
  delete h;
  return MRAFT_OK;
}

int mraft_set_stream(mraft_engine *h, void *stream) {
  if (!h) return fail(MRAFT_E_INVAL, "null engine handle");
  HIP_TRY(hipSetDevice(h->device));
  const hipStream_t ns = stream ? (hipStream_t)stream : (h->tick_masked ? h->tick_masked : h->own_stream);
  // outstanding shard ticks, then everything on the old stream (the engine's
  // stream-ordered buffers may still be in use there), are ordered before the
  // new stream's work: device-side waits, no host wait
  TRY(join_shards(h));
  if (ns != h->stream) {
    hipEvent_t ev = nullptr;
    HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const hipError_t e1 = hipEventRecord(ev, h->stream);
    const hipError_t e2 = e1 == hipSuccess ? hipStreamWaitEvent(ns, ev, 0) : e1;
    (void)hipEventDestroy(ev);  // released once the wait is satisfied
    if (e2 != hipSuccess) return fail(MRAFT_E_HIP, "ordering the new stream: %s", hipGetErrorString(e2));
  }
  h->stream = ns;
  return MRAFT_OK;
}

// With tick shards, the engine stream is first ordered after the outstanding
// shard launches (a device-side wait), so work the caller puts on the returned
// stream sees the tick's outputs. NULL when that ordering fails
// (mraft_last_error_string says why): the stream would not see the outputs.
void *mraft_get_stream(mraft_engine *h) {
  if (!h) {
    fail(MRAFT_E_INVAL, "null engine handle");
    return nullptr;
  }
  if (h->shards_pending) {
    if (hipSetDevice(h->device) != hipSuccess) {
      fail(MRAFT_E_HIP, "hipSetDevice failed");
      return nullptr;
    }
    if (join_shards(h) != MRAFT_OK) return nullptr;
  }
  return (void *)h->stream;
}

int mraft_synchronize(mraft_engine *h) {
  if (!h) return fail(MRAFT_E_INVAL, "null engine handle");
  HIP_TRY(hipSetDevice(h->device));
  TRY(join_shards(h));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return MRAFT_OK;
}

int mraft_dims(const mraft_engine *h, int32_t *g, int32_t *p, int32_t *l) {
  if (!h) return fail(MRAFT_E_INVAL, "null engine handle");
  if (g) *g = h->G;
  if (p) *p = h->P;
  if (l) *l = h->L;
  return MRAFT_OK;
}

int mraft_load_state(mraft_engine *h, const mraft_soa *src, int32_t where) {
  TRY(enter(h));
  if (!src) return fail(MRAFT_E_INVAL, "src is null");
  HIP_TRY(hipSetDevice(h->device));
  const hipMemcpyKind k = where == MRAFT_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
  for (const auto &a : kArrays)
    if (!(src->*(a.ptr))) return fail(MRAFT_E_INVAL, "load_state: every array is required");
  for (const auto &a : kArrays)
    HIP_TRY(hipMemcpyAsync(h->dev.*(a.ptr), src->*(a.ptr), arr_bytes(h, a.kind), k, h->stream));
  mraft::launch_terms_sorted(dev_of(h), h->stream);  // the engine's own proof, not the source's claim
  HIP_TRY(hipGetLastError());
  if (where == MRAFT_HOST) HIP_TRY(hipStreamSynchronize(h->stream));
  return MRAFT_OK;
}

int mraft_store_state(mraft_engine *h, const mraft_soa *dst, int32_t where) {
  TRY(enter(h));
  if (!dst) return fail(MRAFT_E_INVAL, "dst is null");
  HIP_TRY(hipSetDevice(h->device));
  const hipMemcpyKind k = where == MRAFT_HOST ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
  for (const auto &a : kArrays)
    if (dst->*(a.ptr))
      HIP_TRY(hipMemcpyAsync(dst->*(a.ptr), h->dev.*(a.ptr), arr_bytes(h, a.kind), k, h->stream));
  if (where == MRAFT_HOST) HIP_TRY(hipStreamSynchronize(h->stream));
  return MRAFT_OK;
}

int mraft_state_view(mraft_engine *h, mraft_soa *out) {
  TRY(enter(h));
  if (!out) return fail(MRAFT_E_INVAL, "out is null");
  *out = h->dev;
  return MRAFT_OK;
}

int mraft_bind_state(mraft_engine *h, const mraft_soa *d) {
  if (!h) return fail(MRAFT_E_INVAL, "null engine handle");
  if (!d) return fail(MRAFT_E_INVAL, "state is null");
  for (const auto &a : kArrays)
    if (!(d->*(a.ptr))) return fail(MRAFT_E_INVAL, "bind_state: every array is required");
  if (h->owned) {
    drain(h);
    free_owned(h);
  }
  h->dev = *d;
  h->bound = true;
  return MRAFT_OK;
}

// ---------------------------------------------------------------- hot path

// The ticks do not join earlier shard launches (launch_tick forks from the
// engine stream instead): with tick shards, shard s's tick follows its own
// previous tick only. A host-buffer tick joins them before its copies back.
int mraft_replicate_tick(mraft_engine *h, const int32_t *leader_peer, int32_t *group_flags,
                         int32_t where) {
  TRY(check(h));
  if (!leader_peer) return fail(MRAFT_E_INVAL, "leader_peer is null");
  HIP_TRY(hipSetDevice(h->device));
  Stage sg(h, where);
  void *lp, *gf;
  TRY(sg.map(leader_peer, sizeof(int32_t) * h->G, true, false, &lp));
  TRY(sg.map(group_flags, sizeof(int32_t) * h->G, false, true, &gf));
  TRY(launch_tick(h, (const int32_t *)lp, (int32_t *)gf, nullptr, nullptr));
  if (where == MRAFT_HOST) TRY(join_shards(h));
  return sg.finish();
}

int mraft_start_and_tick(mraft_engine *h, const int32_t *leader_peer, const int32_t *counts, int32_t *out_index,
                         int32_t *out_term, int32_t *out_is_leader, int32_t *item_err, int32_t *group_flags,
                         int32_t where) {
  TRY(check(h));
  if (!leader_peer || !counts || !out_index || !out_term || !out_is_leader || !item_err)
    return fail(MRAFT_E_INVAL, "null argument");
  HIP_TRY(hipSetDevice(h->device));
  Stage sg(h, where);
  void *lp, *c, *oi, *ot, *ol, *e, *gf;
  const size_t gb = sizeof(int32_t) * h->G;
  TRY(sg.map(leader_peer, gb, true, false, &lp));
  TRY(sg.map(counts, gb, true, false, &c));
  TRY(sg.map(out_index, gb, false, true, &oi));
  TRY(sg.map(out_term, gb, false, true, &ot));
  TRY(sg.map(out_is_leader, gb, false, true, &ol));
  TRY(sg.map(item_err, gb, false, true, &e));
  TRY(sg.map(group_flags, gb, false, true, &gf));
  const mraft::StartIO sio{(const int32_t *)c, (int32_t *)oi, (int32_t *)ot, (int32_t *)ol, (int32_t *)e};
  TRY(launch_tick(h, (const int32_t *)lp, (int32_t *)gf, nullptr, nullptr, &sio));
  if (where == MRAFT_HOST) TRY(join_shards(h));
  return sg.finish();
}

int mraft_replicate_tick_export(mraft_engine *h, const int32_t *leader_peer, int32_t *group_flags,
                                int32_t *commit, int32_t *term_leader, int32_t where) {
  TRY(check(h));
  if (!leader_peer || !commit || !term_leader) return fail(MRAFT_E_INVAL, "null argument");
  HIP_TRY(hipSetDevice(h->device));
  Stage sg(h, where);
  void *lp, *gf, *c, *t;
  TRY(sg.map(leader_peer, sizeof(int32_t) * h->G, true, false, &lp));
  TRY(sg.map(group_flags, sizeof(int32_t) * h->G, false, true, &gf));
  TRY(sg.map(commit, sizeof(int32_t) * h->G, false, true, &c));
  TRY(sg.map(term_leader, sizeof(int32_t) * h->G, false, true, &t));
  TRY(launch_tick(h, (const int32_t *)lp, (int32_t *)gf, (int32_t *)c, (int32_t *)t));
  if (where == MRAFT_HOST) TRY(join_shards(h));
  return sg.finish();
}

int mraft_replicate_tick_count(mraft_engine *h, const int32_t *leader_peer, int64_t out_words[3],
                               int32_t where) {
  TRY(enter(h));
  if (!leader_peer || !out_words) return fail(MRAFT_E_INVAL, "null argument");
  HIP_TRY(hipSetDevice(h->device));
  Stage sg(h, where);
  void *lp, *cnt;
  TRY(sg.map(leader_peer, sizeof(int32_t) * h->G, true, false, &lp));
  constexpr size_t cw = (size_t)mraft::kCountStripes * mraft::kCountWords;
  TRY(scratch(h, 0, cw * sizeof(unsigned long long), &cnt));
  HIP_TRY(hipMemsetAsync(cnt, 0, cw * sizeof(unsigned long long), h->stream));
  mraft::launch_replicate_tick_count(dev_of(h), (const int32_t *)lp, (unsigned long long *)cnt,
                                     h->stream);
  HIP_TRY(hipGetLastError());
  std::vector<unsigned long long> hc(cw);
  HIP_TRY(hipMemcpyAsync(hc.data(), cnt, cw * sizeof(unsigned long long), hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  for (int i = 0; i < 3; ++i) {
    unsigned long long t = 0;
    for (int x = 0; x < mraft::kCountStripes; ++x) t += hc[(size_t)x * mraft::kCountWords + i];
    out_words[i] = (int64_t)t;
  }
  return MRAFT_OK;
}

int mraft_gather_append_args(mraft_engine *h, const int32_t *slots, const int32_t *peers,
                             int64_t n, mraft_ae_args *out_args, int32_t *item_err, int32_t where) {
  TRY(enter(h));
  if (n < 0 || (n > 0 && (!slots || !peers || !out_args || !item_err)))
    return fail(MRAFT_E_INVAL, "null argument");
  if (n == 0) return MRAFT_OK;
  HIP_TRY(hipSetDevice(h->device));
  Stage sg(h, where);
  void *s, *p, *o, *e;
  TRY(sg.map(slots, sizeof(int32_t) * n, true, false, &s));
  TRY(sg.map(peers, sizeof(int32_t) * n, true, false, &p));
  TRY(sg.map(out_args, sizeof(mraft_ae_args) * n, false, true, &o));
  TRY(sg.map(item_err, sizeof(int32_t) * n, false, true, &e));
  mraft::launch_gather_args(dev_of(h), (const int32_t *)s, (const int32_t *)p, n,
                            (mraft_ae_args *)o, (int32_t *)e, h->stream);
  return sg.finish();
}

int mraft_handle_append_entries(mraft_engine *h, const mraft_ae_args *args, int64_t n,
                                const int32_t *entry_terms, int64_t n_entry_terms,
                                mraft_ae_reply *replies, int32_t *item_err, int32_t where) {
  return mraft_handle_append_entries_ex(h, args, n, entry_terms, n_entry_terms, replies, nullptr, item_err, where);
}

int mraft_handle_append_entries_ex(mraft_engine *h, const mraft_ae_args *args, int64_t n,
                                   const int32_t *entry_terms, int64_t n_entry_terms,
                                   mraft_ae_reply *replies, mraft_ae_result *results, int32_t *item_err,
                                   int32_t where) {
  TRY(enter(h));
  if (n < 0 || (n > 0 && (!args || !replies || !item_err)))
    return fail(MRAFT_E_INVAL, "null argument");
  // item indices are 32-bit in the claims and the ordered fallback
  if (n > INT32_MAX) return fail(MRAFT_E_INVAL, "n = %lld items exceeds 2^31 - 1", (long long)n);
  if (entry_terms && n_entry_terms < 0) return fail(MRAFT_E_INVAL, "n_entry_terms < 0");
  if (n == 0) return MRAFT_OK;
  HIP_TRY(hipSetDevice(h->device));
  TRY(ensure_claim(h));
  Stage sg(h, where);
  void *a, *en, *r, *e, *rs;
  TRY(sg.map(args, sizeof(mraft_ae_args) * n, true, false, &a));
  TRY(sg.map(entry_terms, sizeof(int32_t) * (size_t)(entry_terms ? n_entry_terms : 0), true, false,
             &en));
  TRY(sg.map(replies, sizeof(mraft_ae_reply) * n, false, true, &r));
  TRY(sg.map(results, sizeof(mraft_ae_result) * n, false, true, &rs));
  TRY(sg.map(item_err, sizeof(int32_t) * n, false, true, &e));
  if (en) {  // entries in a caller buffer: one message per wave, nothing is read while written
    mraft::launch_claim(a, n, sizeof(mraft_ae_args), offsetof(mraft_ae_args, slot), nullptr, gp_of(h), h->P,
                        h->claim, h->epoch, (int32_t *)e, h->stream);
    mraft::launch_handle_ae_host(dev_of(h), (const mraft_ae_args *)a, n, (const int32_t *)en, n_entry_terms,
                                 (mraft_ae_reply *)r, (int32_t *)e, (mraft_ae_result *)rs, h->stream);
    return sg.finish();
  }
  // Entries by reference into the engine's log: the claims with the set
  // heads, the main launch, the deferred launch — three launches, every count
  // they need stays on the device, nothing waits on the host (mraft_kernels.hip
  // "a4" for the rules).
  if (!h->ae_total) {
    void *t = nullptr;
    TRY(alloc_async(h, &t, mraft::kAeTotalWords * sizeof(unsigned long long), "AppendEntries counters"));
    h->ae_total = (unsigned long long *)t;
    HIP_TRY(hipMemsetAsync(h->ae_total, 0, mraft::kAeTotalWords * sizeof(unsigned long long), h->stream));
  }
  void *sethd, *soff, *defer, *order, *stage = nullptr;
  TRY(scratch(h, 14, sizeof(int64_t) * (size_t)n, &soff));
  TRY(scratch(h, 15, (size_t)n, &sethd));
  TRY(scratch(h, 18, sizeof(int64_t) * (size_t)n * mraft::kAeStripes, &defer));  // a list of n per stripe
  // the deferred launch's grid: the last call's deferred count (a pinned word
  // the device writes; a stale value only changes the grid, never a result)
  const long long last_nd = *(volatile long long *)h->dhint;
  mraft::AeDeferBufs db{};
  const long long gmin = h->defer_grid_min;
  db.grid = (int)(last_nd < gmin ? gmin : last_nd > kDeferGridMax ? kDeferGridMax : last_nd);
  db.nslot = (int)std::min<int64_t>(db.grid, std::max<int64_t>(1, kCycSlotWords / h->L));
  // the fallback's per-item records and reader counts, its L-word buffer and
  // nslot cycle buffers
  const size_t nn = (size_t)n, L = (size_t)h->L;
  TRY(scratch(h, 19, nn * 16 + (1 + (size_t)db.nslot) * L * 4, &order));
  void *kin = nullptr;
  TRY(scratch_zeroed(h, 20, nn * 8, &kin));  // epoch-tagged: a buffer of its own, zeroed when new
  db.fb = (int4 *)order;
  db.kin = (unsigned long long *)kin;
  db.cyc = (int32_t *)(db.fb + nn);
  db.cslot = db.cyc + L;
  db.hint = h->dhint_dev;
  // MRAFT_STAGE_AUTO: a batch that exceeded the stage (its need published by
  // the device, dhint[1]) grows it for the calls after it (stream-ordered)
  if (h->stage_auto) {
    const long long need = ((volatile long long *)h->dhint)[1];
    if (need > h->stage_cap) {
      const int64_t want = std::min<int64_t>((int64_t)INT32_MAX, (need + need / 4 + kStageStep - 1) / kStageStep * kStageStep);
      h->stage_cap = want;
    }
  }
  // the stage: when it cannot be allocated the batch runs with none (every
  // staged item then takes the ordered fallback: the same results, slower);
  // an automatic stage stops growing there
  if (h->stage_cap > 0 && scratch(h, 16, sizeof(int32_t) * (size_t)h->stage_cap, &stage) != MRAFT_OK) {
    stage = nullptr;
    h->stage_auto = false;
  }
  const int ni = h->P - 1 < 1 ? 1 : h->P - 1 > 7 ? 7 : h->P - 1;
  const int64_t n_log = gp_of(h) * h->L;
  mraft::launch_claim_ae((const mraft_ae_args *)a, n, n_log, h->L, gp_of(h), ni, h->claim, h->srcmark, h->epoch,
                         (int32_t *)e, (uint8_t *)sethd, h->ae_total, h->stream);
  mraft::launch_handle_ae_ref(dev_of(h), (const mraft_ae_args *)a, n, ni, h->claim, h->srcmark, h->epoch,
                              (int32_t *)e, (const uint8_t *)sethd, (int64_t *)soff, (int64_t *)defer, h->ae_total,
                              (int32_t *)stage, stage ? h->stage_cap : 0, db, (mraft_ae_reply *)r,
                              (mraft_ae_result *)rs, h->stream);
  return sg.finish();
}

int mraft_set_stage_capacity(mraft_engine *h, int64_t words) {
  TRY(enter(h));
  if (words == MRAFT_STAGE_AUTO) {
    h->stage_auto = true;
    return MRAFT_OK;
  }
  if (words < 0 || words > INT32_MAX) return fail(MRAFT_E_INVAL, "stage capacity %lld out of [0, 2^31)", (long long)words);
  h->stage_cap = words;
  h->stage_auto = false;
  return MRAFT_OK;
}

int64_t mraft_get_stage_capacity(const mraft_engine *h) { return h ? h->stage_cap : -1; }

int mraft_process_append_replies(mraft_engine *h, const mraft_ae_result *items, int64_t n,
                                 const int64_t *seg_begin, int64_t n_seg, int32_t *out_flags,
                                 int32_t *item_err, int32_t where) {
  TRY(enter(h));
  if (n < 0 || (n > 0 && (!items || !out_flags || !item_err)))
    return fail(MRAFT_E_INVAL, "null argument");
  if (seg_begin && n_seg < 0) return fail(MRAFT_E_INVAL, "n_seg < 0");
  if (n == 0) return MRAFT_OK;
  const int64_t ns = seg_begin ? n_seg : n;
  HIP_TRY(hipSetDevice(h->device));
  TRY(ensure_claim(h));
  Stage sg(h, where);
  void *it, *sb, *fl, *e, *se;
  TRY(sg.map(items, sizeof(mraft_ae_result) * n, true, false, &it));
  TRY(sg.map(seg_begin, sizeof(int64_t) * (size_t)(seg_begin ? n_seg + 1 : 0), true, false, &sb));
  TRY(sg.map(out_flags, sizeof(int32_t) * n, false, true, &fl));
  TRY(sg.map(item_err, sizeof(int32_t) * n, false, true, &e));
  TRY(scratch(h, 1, sizeof(int32_t) * (size_t)ns, &se));
  void *sc;
  TRY(scratch(h, 7, mraft::fold_scan_bytes(n, ns), &sc));
  // three launches: the segment claims with the outputs zeroed, the fold
  // (which rejects a segment whose slot another one claimed), the tail (the
  // segments longer than a lane group, and the a1 scans the probes left open)
  mraft::launch_fold(dev_of(h), (const mraft_ae_result *)it, n, (const int64_t *)sb, ns, gp_of(h), h->claim,
                     h->epoch, (int32_t *)se, (int32_t *)fl, (int32_t *)e, sc, h->stream);
  return sg.finish();
}

int mraft_start(mraft_engine *h, const int32_t *slots, const int32_t *counts, int64_t n,
                int32_t *out_index, int32_t *out_term, int32_t *out_is_leader, int32_t *item_err,
                int32_t where) {
  TRY(enter(h));
  if (n < 0 || (n > 0 && (!slots || !out_index || !out_term || !out_is_leader || !item_err)))
    return fail(MRAFT_E_INVAL, "null argument");
  if (n == 0) return MRAFT_OK;
  HIP_TRY(hipSetDevice(h->device));
  TRY(ensure_claim(h));
  Stage sg(h, where);
  void *s, *c, *oi, *ot, *ol, *e;
  TRY(sg.map(slots, sizeof(int32_t) * n, true, false, &s));
  TRY(sg.map(counts, sizeof(int32_t) * n, true, false, &c));
  TRY(sg.map(out_index, sizeof(int32_t) * n, false, true, &oi));
  TRY(sg.map(out_term, sizeof(int32_t) * n, false, true, &ot));
  TRY(sg.map(out_is_leader, sizeof(int32_t) * n, false, true, &ol));
  TRY(sg.map(item_err, sizeof(int32_t) * n, false, true, &e));
  mraft::launch_start(dev_of(h), (const int32_t *)s, (const int32_t *)c, n, (int32_t *)oi,
                      (int32_t *)ot, (int32_t *)ol, (int32_t *)e, h->claim, h->epoch, h->stream);
  return sg.finish();
}

int mraft_collect_apply(mraft_engine *h, int32_t *out_from, int32_t *out_to, int32_t *out_snap_index,
                        int32_t *out_snap_term, int32_t where) {
  TRY(enter(h));
  if (!out_from || !out_to) return fail(MRAFT_E_INVAL, "null argument");
  if (!out_snap_index != !out_snap_term) return fail(MRAFT_E_INVAL, "snapshot outputs: both or neither");
  HIP_TRY(hipSetDevice(h->device));
  Stage sg(h, where);
  void *f, *t, *si, *st;
  TRY(sg.map(out_from, sizeof(int32_t) * gp_of(h), false, true, &f));
  TRY(sg.map(out_to, sizeof(int32_t) * gp_of(h), false, true, &t));
  TRY(sg.map(out_snap_index, sizeof(int32_t) * gp_of(h), false, true, &si));
  TRY(sg.map(out_snap_term, sizeof(int32_t) * gp_of(h), false, true, &st));
  mraft::launch_collect_apply(dev_of(h), (int32_t *)f, (int32_t *)t, (int32_t *)si, (int32_t *)st, h->stream);
  return sg.finish();
}

int mraft_collect_apply_compact(mraft_engine *h, int32_t *out_slots, int32_t *out_snap_index,
                                int32_t *out_snap_term, int32_t *out_from, int32_t *out_to, int64_t cap,
                                int64_t *out_n, int32_t where) {
  TRY(enter(h));
  if (cap < 0 || !out_n || (cap > 0 && (!out_slots || !out_from || !out_to)) ||
      (!out_snap_index) != (!out_snap_term))
    return fail(MRAFT_E_INVAL, "null argument");
  HIP_TRY(hipSetDevice(h->device));
  Stage sg(h, where);
  void *sl, *si, *stm, *f, *t, *n, *bc;
  TRY(sg.map(out_slots, sizeof(int32_t) * (size_t)cap, false, true, &sl));
  TRY(sg.map(out_snap_index, sizeof(int32_t) * (size_t)cap, false, true, &si));
  TRY(sg.map(out_snap_term, sizeof(int32_t) * (size_t)cap, false, true, &stm));
  TRY(sg.map(out_from, sizeof(int32_t) * (size_t)cap, false, true, &f));
  TRY(sg.map(out_to, sizeof(int32_t) * (size_t)cap, false, true, &t));
  TRY(sg.map(out_n, sizeof(int64_t), false, true, &n));
  TRY(scratch(h, 6, sizeof(int32_t) * (size_t)((gp_of(h) + 255) / 256), &bc));
  mraft::launch_collect_apply_compact(dev_of(h), (int32_t *)bc, cap, (int32_t *)sl, (int32_t *)si,
                                      (int32_t *)stm, (int32_t *)f, (int32_t *)t, (int64_t *)n, h->stream);
  return sg.finish();
}

int mraft_snapshot(mraft_engine *h, const int32_t *slots, const int32_t *index, int64_t n,
                   int32_t *item_err, int32_t where) {
  TRY(enter(h));
  if (n < 0 || (n > 0 && (!slots || !index || !item_err))) return fail(MRAFT_E_INVAL, "null argument");
  if (n == 0) return MRAFT_OK;
  HIP_TRY(hipSetDevice(h->device));
  TRY(ensure_claim(h));
  Stage sg(h, where);
  void *s, *x, *e;
  TRY(sg.map(slots, sizeof(int32_t) * n, true, false, &s));
  TRY(sg.map(index, sizeof(int32_t) * n, true, false, &x));
  TRY(sg.map(item_err, sizeof(int32_t) * n, false, true, &e));
  mraft::launch_claim(s, n, sizeof(int32_t), 0, nullptr, gp_of(h), h->P, h->claim, h->epoch,
                      (int32_t *)e, h->stream);
  mraft::launch_snapshot(dev_of(h), (const int32_t *)s, (const int32_t *)x, n, (int32_t *)e, h->stream);
  return sg.finish();
}

int mraft_gather_install_snapshot_args(mraft_engine *h, const int32_t *slots, const int32_t *peers,
                                       int64_t n, mraft_is_args *out_args, int32_t *item_err,
                                       int32_t where) {
  TRY(enter(h));
  if (n < 0 || (n > 0 && (!slots || !peers || !out_args || !item_err)))
    return fail(MRAFT_E_INVAL, "null argument");
  if (n == 0) return MRAFT_OK;
  HIP_TRY(hipSetDevice(h->device));
  Stage sg(h, where);
  void *s, *p, *o, *e;
  TRY(sg.map(slots, sizeof(int32_t) * n, true, false, &s));
  TRY(sg.map(peers, sizeof(int32_t) * n, true, false, &p));
  TRY(sg.map(out_args, sizeof(mraft_is_args) * n, false, true, &o));
  TRY(sg.map(item_err, sizeof(int32_t) * n, false, true, &e));
  mraft::launch_gather_is(dev_of(h), (const int32_t *)s, (const int32_t *)p, n, (mraft_is_args *)o,
                          (int32_t *)e, h->stream);
  return sg.finish();
}

int mraft_handle_install_snapshot(mraft_engine *h, const mraft_is_args *args, int64_t n,
                                  mraft_is_reply *replies, int32_t *out_flags, int32_t *item_err,
                                  int32_t where) {
  TRY(enter(h));
  if (n < 0 || (n > 0 && (!args || !replies || !out_flags || !item_err)))
    return fail(MRAFT_E_INVAL, "null argument");
  if (n == 0) return MRAFT_OK;
  HIP_TRY(hipSetDevice(h->device));
  TRY(ensure_claim(h));
  Stage sg(h, where);
  void *a, *r, *f, *e;
  TRY(sg.map(args, sizeof(mraft_is_args) * n, true, false, &a));
  TRY(sg.map(replies, sizeof(mraft_is_reply) * n, false, true, &r));
  TRY(sg.map(out_flags, sizeof(int32_t) * n, false, true, &f));
  TRY(sg.map(item_err, sizeof(int32_t) * n, false, true, &e));
  mraft::launch_claim(a, n, sizeof(mraft_is_args), offsetof(mraft_is_args, slot), nullptr, gp_of(h),
                      h->P, h->claim, h->epoch, (int32_t *)e, h->stream);
  mraft::launch_handle_is(dev_of(h), (const mraft_is_args *)a, n, (mraft_is_reply *)r, (int32_t *)f,
                          (int32_t *)e, h->stream);
  return sg.finish();
}

int mraft_process_install_snapshot_replies(mraft_engine *h, const mraft_is_result *items, int64_t n,
                                           const int64_t *seg_begin, int64_t n_seg,
                                           int32_t *out_flags, int32_t *item_err, int32_t where) {
  TRY(enter(h));
  if (n < 0 || (n > 0 && (!items || !out_flags || !item_err)))
    return fail(MRAFT_E_INVAL, "null argument");
  if (seg_begin && n_seg < 0) return fail(MRAFT_E_INVAL, "n_seg < 0");
  if (n == 0) return MRAFT_OK;
  const int64_t ns = seg_begin ? n_seg : n;
  HIP_TRY(hipSetDevice(h->device));
  TRY(ensure_claim(h));
  Stage sg(h, where);
  void *it, *sb, *fl, *e, *se;
  TRY(sg.map(items, sizeof(mraft_is_result) * n, true, false, &it));
  TRY(sg.map(seg_begin, sizeof(int64_t) * (size_t)(seg_begin ? n_seg + 1 : 0), true, false, &sb));
  TRY(sg.map(out_flags, sizeof(int32_t) * n, false, true, &fl));
  TRY(sg.map(item_err, sizeof(int32_t) * n, false, true, &e));
  TRY(scratch(h, 1, sizeof(int32_t) * (size_t)ns, &se));
  HIP_TRY(hipMemsetAsync(fl, 0, sizeof(int32_t) * n, h->stream));
  HIP_TRY(hipMemsetAsync(e, 0, sizeof(int32_t) * n, h->stream));
  mraft::launch_claim(it, ns, sizeof(mraft_is_result), offsetof(mraft_is_result, slot),
                      (const int64_t *)sb, gp_of(h), h->P, h->claim, h->epoch, (int32_t *)se,
                      h->stream);
  mraft::launch_process_is(dev_of(h), (const mraft_is_result *)it, n, (const int64_t *)sb, ns,
                           (int32_t *)se, (int32_t *)fl, (int32_t *)e, h->stream);
  return sg.finish();
}

int mraft_start_election(mraft_engine *h, const int32_t *slots, int64_t n, mraft_rv_args *out_args,
                         int32_t *item_err, int32_t where) {
  TRY(enter(h));
  if (n < 0 || (n > 0 && (!slots || !out_args || !item_err)))
    return fail(MRAFT_E_INVAL, "null argument");
  if (n == 0) return MRAFT_OK;
  HIP_TRY(hipSetDevice(h->device));
  TRY(ensure_claim(h));
  Stage sg(h, where);
  void *s, *o, *e;
  TRY(sg.map(slots, sizeof(int32_t) * n, true, false, &s));
  TRY(sg.map(out_args, sizeof(mraft_rv_args) * n, false, true, &o));
  TRY(sg.map(item_err, sizeof(int32_t) * n, false, true, &e));
  mraft::launch_claim(s, n, sizeof(int32_t), 0, nullptr, gp_of(h), h->P, h->claim, h->epoch,
                      (int32_t *)e, h->stream);
  mraft::launch_start_election(dev_of(h), (const int32_t *)s, n, (mraft_rv_args *)o, (int32_t *)e,
                               h->stream);
  return sg.finish();
}

int mraft_handle_request_vote(mraft_engine *h, const mraft_rv_args *args, int64_t n,
                              mraft_rv_reply *replies, int32_t *item_err, int32_t where) {
  TRY(enter(h));
  if (n < 0 || (n > 0 && (!args || !replies || !item_err)))
    return fail(MRAFT_E_INVAL, "null argument");
  if (n == 0) return MRAFT_OK;
  HIP_TRY(hipSetDevice(h->device));
  TRY(ensure_claim(h));
  Stage sg(h, where);
  void *a, *r, *e;
  TRY(sg.map(args, sizeof(mraft_rv_args) * n, true, false, &a));
  TRY(sg.map(replies, sizeof(mraft_rv_reply) * n, false, true, &r));
  TRY(sg.map(item_err, sizeof(int32_t) * n, false, true, &e));
  mraft::launch_claim(a, n, sizeof(mraft_rv_args), offsetof(mraft_rv_args, slot), nullptr, gp_of(h),
                      h->P, h->claim, h->epoch, (int32_t *)e, h->stream);
  mraft::launch_handle_rv(dev_of(h), (const mraft_rv_args *)a, n, (mraft_rv_reply *)r, (int32_t *)e,
                          h->stream);
  return sg.finish();
}

int mraft_process_vote_replies(mraft_engine *h, const mraft_rv_result *items, int64_t n,
                               const int64_t *seg_begin, int64_t n_seg, int32_t *out_flags,
                               int32_t *item_err, int32_t where) {
  TRY(enter(h));
  if (n < 0 || (n > 0 && (!items || !out_flags || !item_err)))
    return fail(MRAFT_E_INVAL, "null argument");
  if (seg_begin && n_seg < 0) return fail(MRAFT_E_INVAL, "n_seg < 0");
  if (n == 0) return MRAFT_OK;
  const int64_t ns = seg_begin ? n_seg : n;
  HIP_TRY(hipSetDevice(h->device));
  TRY(ensure_claim(h));
  Stage sg(h, where);
  void *it, *sb, *fl, *e, *se;
  TRY(sg.map(items, sizeof(mraft_rv_result) * n, true, false, &it));
  TRY(sg.map(seg_begin, sizeof(int64_t) * (size_t)(seg_begin ? n_seg + 1 : 0), true, false, &sb));
  TRY(sg.map(out_flags, sizeof(int32_t) * n, false, true, &fl));
  TRY(sg.map(item_err, sizeof(int32_t) * n, false, true, &e));
  TRY(scratch(h, 1, sizeof(int32_t) * (size_t)ns, &se));
  HIP_TRY(hipMemsetAsync(fl, 0, sizeof(int32_t) * n, h->stream));
  HIP_TRY(hipMemsetAsync(e, 0, sizeof(int32_t) * n, h->stream));
  mraft::launch_claim(it, ns, sizeof(mraft_rv_result), offsetof(mraft_rv_result, slot),
                      (const int64_t *)sb, gp_of(h), h->P, h->claim, h->epoch, (int32_t *)se,
                      h->stream);
  mraft::launch_tally(dev_of(h), (const mraft_rv_result *)it, n, (const int64_t *)sb, ns,
                      (int32_t *)se, (int32_t *)fl, (int32_t *)e, h->stream);
  return sg.finish();
}

int mraft_election_rounds(mraft_engine *h, const uint8_t *cand_mask, int32_t rounds,
                          int32_t *group_flags, int32_t where) {
  TRY(enter(h));
  if (!cand_mask || rounds < 0) return fail(MRAFT_E_INVAL, "null mask or negative rounds");
  HIP_TRY(hipSetDevice(h->device));
  Stage sg(h, where);
  void *m, *gf;
  TRY(sg.map(cand_mask, (size_t)rounds * h->G, true, false, &m));
  TRY(sg.map(group_flags, sizeof(int32_t) * h->G, false, true, &gf));
  mraft::launch_election_rounds(dev_of(h), (const uint8_t *)m, rounds, (int32_t *)gf, h->stream);
  return sg.finish();
}

// ---------------------------------------------------------------- persistence

int mraft_collect_persist(mraft_engine *h, int32_t *out_bits, int32_t where) {
  TRY(enter(h));
  if (!out_bits) return fail(MRAFT_E_INVAL, "out_bits is null");
  HIP_TRY(hipSetDevice(h->device));
  Stage sg(h, where);
  void *o;
  TRY(sg.map(out_bits, sizeof(int32_t) * (size_t)gp_of(h), false, true, &o));
  mraft::launch_collect_persist(dev_of(h), (int32_t *)o, h->stream);
  return sg.finish();
}

int mraft_read_persistent(mraft_engine *h, const int32_t *slots, int64_t n, mraft_persistent *out,
                          int32_t *out_terms, int64_t terms_cap) {
  TRY(enter(h));
  if (n < 0 || (n > 0 && (!slots || !out))) return fail(MRAFT_E_INVAL, "null argument");
  if (n == 0) return MRAFT_OK;
  for (int64_t i = 0; i < n; ++i)
    if (slots[i] < 0 || slots[i] >= gp_of(h)) return fail(MRAFT_E_INVAL, "slot %d out of range", slots[i]);
  HIP_TRY(hipSetDevice(h->device));
  void *ds, *dh, *dt;
  TRY(scratch(h, 2, sizeof(int32_t) * (size_t)n, &ds));
  TRY(scratch(h, 3, sizeof(mraft_persistent) * (size_t)n, &dh));
  HIP_TRY(hipMemcpyAsync(ds, slots, sizeof(int32_t) * n, hipMemcpyHostToDevice, h->stream));
  mraft::launch_read_persistent_hdr(dev_of(h), (const int32_t *)ds, n, (mraft_persistent *)dh, h->stream);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out, dh, sizeof(mraft_persistent) * n, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  int64_t off = 0;
  for (int64_t i = 0; i < n; ++i) {
    out[i].terms_offset = off;
    off += (int64_t)out[i].last_index - out[i].dummy_index + 1;
  }
  if (!out_terms || terms_cap < off)
    return fail(MRAFT_E_INVAL, "read_persistent: %lld terms needed, capacity %lld", (long long)off,
                (long long)terms_cap);
  TRY(scratch(h, 4, sizeof(int32_t) * (size_t)off, &dt));
  HIP_TRY(hipMemcpyAsync(dh, out, sizeof(mraft_persistent) * n, hipMemcpyHostToDevice, h->stream));
  mraft::launch_read_persistent_terms(dev_of(h), (const mraft_persistent *)dh, n, (int32_t *)dt,
                                      h->stream);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out_terms, dt, sizeof(int32_t) * off, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return MRAFT_OK;
}

int mraft_restore(mraft_engine *h, const mraft_persistent *in, int64_t n, const int32_t *terms,
                  int64_t n_terms, int32_t *item_err) {
  TRY(enter(h));
  if (n < 0 || (n > 0 && (!in || !item_err || (n_terms > 0 && !terms))))
    return fail(MRAFT_E_INVAL, "null argument");
  if (n == 0) return MRAFT_OK;
  std::vector<char> seen((size_t)gp_of(h), 0);
  for (int64_t i = 0; i < n; ++i) {
    const mraft_persistent &r = in[i];
    const int64_t cnt = (int64_t)r.last_index - r.dummy_index + 1;
    int e = MRAFT_ITEM_OK;
    if (r.slot < 0 || r.slot >= gp_of(h) || cnt < 1 || r.dummy_index < 0 || r.terms_offset < 0 ||
        r.terms_offset + cnt > n_terms)
      e = MRAFT_ITEM_BAD_SLOT;
    else if (cnt > h->L)
      e = MRAFT_ITEM_LOG_FULL;
    else if (seen[(size_t)r.slot])
      e = MRAFT_ITEM_DUP_SLOT;
    if (e == MRAFT_ITEM_OK) seen[(size_t)r.slot] = 1;
    item_err[i] = e;
  }
  HIP_TRY(hipSetDevice(h->device));
  void *dh, *dt, *de;
  TRY(scratch(h, 3, sizeof(mraft_persistent) * (size_t)n, &dh));
  TRY(scratch(h, 4, sizeof(int32_t) * (size_t)(n_terms > 0 ? n_terms : 1), &dt));
  TRY(scratch(h, 5, sizeof(int32_t) * (size_t)n, &de));
  HIP_TRY(hipMemcpyAsync(dh, in, sizeof(mraft_persistent) * n, hipMemcpyHostToDevice, h->stream));
  if (n_terms > 0)
    HIP_TRY(hipMemcpyAsync(dt, terms, sizeof(int32_t) * n_terms, hipMemcpyHostToDevice, h->stream));
  HIP_TRY(hipMemcpyAsync(de, item_err, sizeof(int32_t) * n, hipMemcpyHostToDevice, h->stream));
  mraft::launch_restore(dev_of(h), (const mraft_persistent *)dh, n, (const int32_t *)dt,
                        (const int32_t *)de, h->stream);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(h->stream));
  return MRAFT_OK;
}

int mraft_export_group_status(mraft_engine *h, const int32_t *leader_peer, int32_t *commit,
                              int32_t *term_leader, int32_t where) {
  TRY(enter(h));
  if (!commit || !term_leader) return fail(MRAFT_E_INVAL, "null argument");
  HIP_TRY(hipSetDevice(h->device));
  Stage sg(h, where);
  void *lp, *c, *t;
  TRY(sg.map(leader_peer, sizeof(int32_t) * h->G, true, false, &lp));
  TRY(sg.map(commit, sizeof(int32_t) * h->G, false, true, &c));
  TRY(sg.map(term_leader, sizeof(int32_t) * h->G, false, true, &t));
  mraft::launch_export(dev_of(h), (const int32_t *)lp, (int32_t *)c, (int32_t *)t, h->stream);
  return sg.finish();
}

}  // extern "C"

// ---------------------------------------------------------------- fan-in (§8e)

namespace {

#define NCCL_TRY(expr)                                                                  \
  do {                                                                                  \
    ncclResult_t r_ = (expr);                                                           \
    if (r_ != ncclSuccess)                                                              \
      return fail(MRAFT_E_HIP, "%s failed: %s", #expr, ncclGetErrorString(r_));         \
  } while (0)

int fanin_stream_of(mraft_engine *h, hipStream_t *out) {
  if (h->fanin_masked) {
    *out = h->fanin_masked;
    return MRAFT_OK;
  }
  if (!h->fanin_own) HIP_TRY(hipStreamCreateWithFlags(&h->fanin_own, hipStreamNonBlocking));
  *out = h->fanin_own;
  return MRAFT_OK;
}

}  // namespace

extern "C" {

int mraft_comm_unique_id(uint8_t out[MRAFT_COMM_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) == MRAFT_COMM_ID_BYTES, "RCCL unique id size");
  if (!out) return fail(MRAFT_E_INVAL, "out is null");
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  std::memcpy(out, &id, sizeof id);
  return MRAFT_OK;
}

int mraft_comm_init(mraft_engine *h, int32_t nranks, int32_t rank, const uint8_t id[MRAFT_COMM_ID_BYTES],
                    void **out_comm) {
  if (!h || !id || !out_comm) return fail(MRAFT_E_INVAL, "null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(MRAFT_E_INVAL, "bad rank %d of %d", rank, nranks);
  *out_comm = nullptr;
  HIP_TRY(hipSetDevice(h->device));
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof uid);
  ncclComm_t c = nullptr;
  NCCL_TRY(ncclCommInitRank(&c, nranks, uid, rank));
  *out_comm = (void *)c;
  return MRAFT_OK;
}

int mraft_comm_destroy(void *comm) {
  if (!comm) return MRAFT_OK;
  NCCL_TRY(ncclCommDestroy((ncclComm_t)comm));
  return MRAFT_OK;
}

int mraft_allgather_status(mraft_engine *h, void *comm, const int32_t *local, int32_t *gathered,
                           int32_t where, uint32_t flags) {
  if (!h) return fail(MRAFT_E_INVAL, "null engine handle");
  if (!comm || !local || !gathered) return fail(MRAFT_E_INVAL, "null argument");
  HIP_TRY(hipSetDevice(h->device));
  // Without OVERLAP/ORDERED the gather runs on the engine stream, after the
  // shard launches (joined). With OVERLAP it waits for them on the fan-in
  // stream only, so the next tick's shards do not wait for this tick's others.
  if (where == MRAFT_HOST || !(flags & (MRAFT_FANIN_OVERLAP | MRAFT_FANIN_ORDERED))) TRY(join_shards(h));
  ncclComm_t c = (ncclComm_t)comm;
  int nranks = 0;
  NCCL_TRY(ncclCommCount(c, &nranks));
  const size_t words = 2 * (size_t)h->G;
  if (where == MRAFT_HOST) {
    Stage sg(h, where);
    void *l, *g;
    TRY(sg.map(local, sizeof(int32_t) * words, true, false, &l));
    TRY(sg.map(gathered, sizeof(int32_t) * words * nranks, false, true, &g));
    NCCL_TRY(ncclAllGather(l, g, words, ncclInt32, c, h->stream));
    return sg.finish();
  }
  hipStream_t st = h->stream;
  if (flags & MRAFT_FANIN_ORDERED) {
    TRY(fanin_stream_of(h, &st));
  } else if (flags & MRAFT_FANIN_OVERLAP) {
    TRY(fanin_stream_of(h, &st));
    if (!h->fanin_ev) HIP_TRY(hipEventCreateWithFlags(&h->fanin_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(h->fanin_ev, h->stream));
    HIP_TRY(hipStreamWaitEvent(st, h->fanin_ev, 0));
    if (h->shards_pending)
      for (int k = 0; k < h->nshards; ++k) {
        HIP_TRY(hipEventRecord(h->shard_ev[k], h->shard_q[k]));
        HIP_TRY(hipStreamWaitEvent(st, h->shard_ev[k], 0));
      }
  }
  NCCL_TRY(ncclAllGather(local, gathered, words, ncclInt32, c, st));
  HIP_TRY(hipGetLastError());
  return MRAFT_OK;
}

int mraft_fanin_synchronize(mraft_engine *h) {
  if (!h) return fail(MRAFT_E_INVAL, "null engine handle");
  HIP_TRY(hipSetDevice(h->device));
  hipStream_t st;
  TRY(fanin_stream_of(h, &st));
  HIP_TRY(hipStreamSynchronize(st));
  return MRAFT_OK;
}

void *mraft_fanin_stream(mraft_engine *h) {
  if (!h) return nullptr;
  hipStream_t st = nullptr;
  if (hipSetDevice(h->device) != hipSuccess || fanin_stream_of(h, &st) != MRAFT_OK) return nullptr;
  return (void *)st;
}

int mraft_fanin_reserve_cus(mraft_engine *h, int32_t n_cus) {
  if (!h) return fail(MRAFT_E_INVAL, "null engine handle");
  HIP_TRY(hipSetDevice(h->device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, h->device));
  const int ncu = prop.multiProcessorCount;
  if (n_cus < 0 || n_cus >= ncu) return fail(MRAFT_E_INVAL, "n_cus %d of %d CUs", n_cus, ncu);
  drain(h);
  for (hipStream_t *s : {&h->fanin_masked, &h->tick_masked})
    if (*s) {
      HIP_TRY(hipStreamSynchronize(*s));
      HIP_TRY(hipStreamDestroy(*s));
      *s = nullptr;
    }
  h->fan_cus = n_cus;
  // tick shards: their queues take the tick side's mask; the engine stream
  // carries no tick and stays as it is
  const int S = h->nshards;
  if (S > 1) {
    destroy_shard_queues(h);
    TRY(create_shard_queues(h, S));
  }
  if (n_cus == 0) {
    if (S <= 1) h->stream = h->own_stream;
    return MRAFT_OK;
  }
  if (S <= 1) {
    TRY(make_queue(h, true, &h->tick_masked));
    h->stream = h->tick_masked;
  }
  TRY(make_queue(h, false, &h->fanin_masked));
  return MRAFT_OK;
}

int mraft_set_tick_shards(mraft_engine *h, int32_t shards) {
  if (!h) return fail(MRAFT_E_INVAL, "null engine handle");
  if (shards < 1 || shards > kMaxShards || shards > h->G)
    return fail(MRAFT_E_INVAL, "shards %d (need 1..%d and at most G = %d)", shards, kMaxShards, h->G);
  HIP_TRY(hipSetDevice(h->device));
  drain(h);
  destroy_shard_queues(h);
  h->nshards = 1;
  if (shards > 1) {
    TRY(create_shard_queues(h, shards));
    h->nshards = shards;
    // the masked tick stream of a one-shard engine (mraft_fanin_reserve_cus)
    // is not needed: the shard queues carry the mask
    if (h->tick_masked) {
      if (h->stream == h->tick_masked) h->stream = h->own_stream;
      HIP_TRY(hipStreamDestroy(h->tick_masked));
      h->tick_masked = nullptr;
    }
  } else if (h->fan_cus > 0 && !h->tick_masked) {
    TRY(make_queue(h, true, &h->tick_masked));
    if (h->stream == h->own_stream) h->stream = h->tick_masked;
  }
  return MRAFT_OK;
}

int32_t mraft_get_tick_shards(const mraft_engine *h) { return h ? h->nshards : 0; }

int mraft_set_tick_mode(mraft_engine *h, int32_t mode) {
  if (!h) return fail(MRAFT_E_INVAL, "null engine handle");
  if (mode != MRAFT_TICK_FULL && mode != MRAFT_TICK_LIGHT && mode != MRAFT_TICK_AUTO)
    return fail(MRAFT_E_INVAL, "tick mode %d", mode);
  h->tick_mode = mode;
  return MRAFT_OK;
}

int32_t mraft_get_tick_mode(const mraft_engine *h) { return h ? h->tick_mode : -1; }

int64_t mraft_tick_light_fallbacks(mraft_engine *h) {
  if (!h) return -1;
  long long t = 0;
  for (int s = 0; s < std::max(1, (int)h->nshards); ++s) {
    const long long v = ((volatile long long *)h->dhint)[kHintLite + s];
    if (v < 0) return -1;
    t += v;
  }
  return t;
}

void *mraft_shard_stream(mraft_engine *h, int32_t shard) {
  if (!h || shard < 0 || shard >= h->nshards) return nullptr;
  return h->nshards > 1 ? (void *)h->shard_q[shard] : (void *)h->stream;
}

}  // extern "C"
