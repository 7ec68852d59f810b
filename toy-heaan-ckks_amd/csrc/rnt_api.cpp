// rnt_api.cpp -- the extern "C" boundary (include/rnsntt.h) over the HIP
// kernels.  Every entry point validates like the reference (errors.rs:4-20
// order), turns every failure into a status code, and never lets a C++
// exception or HIP error escape.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cinttypes>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/rnsntt.h"
#include "rnt_hostmath.hpp"
#include "rnt_internal.hpp"

namespace {

thread_local std::string g_last_error;
// the RnsNttError fields of the last failure (rnt_last_error_detail)
struct ErrDetail {
  int status;
  uint64_t a, b;
};
thread_local ErrDetail g_last_detail{0, 0, 0};

int vfail(int code, uint64_t a, uint64_t b, const char* fmt, va_list ap) {
  char buf[512];
  vsnprintf(buf, sizeof buf, fmt, ap);
  g_last_error = buf;
  g_last_detail = {code, a, b};
  return code;
}

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfail(code, 0, 0, fmt, ap);
  va_end(ap);
  return code;
}

// A failure that carries the reference variant's fields (errors.rs:4-20).
int fail_fields(int code, uint64_t a, uint64_t b, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfail(code, a, b, fmt, ap);
  va_end(ap);
  return code;
}

int hip_fail(hipError_t e, const char* where) {
  (void)hipGetLastError();  // reported here: not pending for the next call
  if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation)
    return fail(RNT_ERR_OUT_OF_MEMORY, "%s: %s", where, hipGetErrorString(e));
  return fail(RNT_ERR_DEVICE, "%s: %s", where, hipGetErrorString(e));
}

#define HIP_TRY(expr, where)                  \
  do {                                        \
    hipError_t e_ = (expr);                   \
    if (e_ != hipSuccess) return hip_fail(e_, where); \
  } while (0)

inline size_t word_bytes(const rnt::Tables* t) { return t->wide ? 8 : 4; }

// An op sequence being recorded into a hipGraph on this thread
// (rnt_capture_begin .. rnt_capture_end): workspace blocks the captured ops
// take stay with the graph, whose replays reuse those exact addresses, and
// nothing that would synchronise the stream runs while recording.
// Only blocks handed back on the recording's own device and stream go to the
// graph (a block freed on another context while recording goes back to the
// cache as usual).  Call-scoped workspace (CallWs) handed back while
// recording is idle again for the next recorded op: `idle` blocks are taken
// before the cache is asked, so N recorded key-switch ops share one
// workspace (the recorded ops are ordered on the one captured stream), and
// the graph keeps the distinct blocks only.
struct OwnedBlock {
  void* p;
  size_t bytes;
  bool idle;
};
struct Capture {
  std::vector<OwnedBlock> owned;
  hipStream_t stream = nullptr;
  int device = 0;
};
thread_local Capture* g_capture = nullptr;

const char* const kKernelNames[rnt::K_COUNT] = {
    "col_fwd", "row_fwd", "row_inv", "row_mul", "col_inv", "elementwise", "rescale",
    "automorphism", "ks_decompose", "ks_rows", "tensor_rows", "import", "export", "crt",
    "sfft", "sample", "copy", "plane_fused", "mf_ntt_fwd", "mf_ntt_inv", "whole_fwd", "whole_inv", "whole_mul", "ks_whole", "tensor_whole", "mf_tensor", "mf_mul"};

// A profiling call failed: clear the runtime's slot, keep the first failure
// in the profiler, and stop profiling (rnt_profile_read reports it).
void prof_fail(rnt::Prof* p, hipError_t e, const char* where) {
  (void)hipGetLastError();
  if (p->err == hipSuccess) {
    p->err = e;
    p->err_where = where;
  }
  p->on = false;
}
hipEvent_t prof_event(rnt::Prof* p) {
  if (!p->pool.empty()) {
    hipEvent_t e = p->pool.back();
    p->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (const hipError_t r = hipEventCreate(&e); r != hipSuccess) {
    prof_fail(p, r, "hipEventCreate(profile)");
    return nullptr;
  }
  return e;
}

// HIP errors are never dropped.  A cleanup call whose failure cannot abort
// the call making it (a block leaving the cache, a destructor, an event
// released) goes through cleanup(): the first such failure on the thread is
// kept with the call's name, and the runtime's last-error slot is cleared.
// The library then reports it as RNT_ERR_DEVICE, naming that call: from the
// entry point that made it when that one returns a status of its own
// (rnt_buf_free, rnt_ctx_destroy, rnt_graph_destroy, rnt_pool_trim), else
// from the next launch on the thread (check_pending).  A launcher reads
// hipGetLastError() after its launch, so an error some other code left in
// the slot would otherwise be blamed on the launch: check_pending reports it
// before launching, as pending from an earlier call, instead of clearing it.
struct Deferred {
  hipError_t e = hipSuccess;
  const char* where = nullptr;
};
thread_local Deferred g_deferred;

inline void cleanup(hipError_t e, const char* where) {
  if (e == hipSuccess) return;
  (void)hipGetLastError();  // kept in g_deferred instead
  if (g_deferred.e == hipSuccess) g_deferred = {e, where};
}

// RNT_OK, or the first deferred cleanup failure of this thread as a status.
int take_deferred() {
  if (g_deferred.e == hipSuccess) return RNT_OK;
  const Deferred d = g_deferred;
  g_deferred = {};
  return fail(RNT_ERR_DEVICE, "%s failed: %s (a cleanup call, reported at the next status)", d.where,
              hipGetErrorString(d.e));
}

// A free / destroy / trim entry point reports only the failures of its own
// cleanup calls: a failure some earlier call deferred stays pending for the
// next launch (check_pending) instead of being consumed -- or blamed on the
// free -- here.  Bindings may drop a free's status (a destructor, __del__);
// an unrelated earlier failure then still reaches a status that is checked.
struct OwnCleanup {
  Deferred saved;
  OwnCleanup() : saved(g_deferred) { g_deferred = {}; }
  int finish() {
    const Deferred mine = g_deferred;
    g_deferred = saved;
    saved = {};
    if (mine.e == hipSuccess) return RNT_OK;
    return fail(RNT_ERR_DEVICE, "%s failed: %s", mine.where, hipGetErrorString(mine.e));
  }
  ~OwnCleanup() {
    if (saved.e != hipSuccess && g_deferred.e == hipSuccess) g_deferred = saved;
  }
};

// Before a launch: a deferred cleanup failure, or an error some earlier
// runtime call on this thread left unreported in the last-error slot.
int check_pending(int id) {
  if (int rc = take_deferred()) return rc;
  const hipError_t pre = hipGetLastError();
  if (pre != hipSuccess)
    return fail(RNT_ERR_DEVICE,
                "a HIP error was pending before the %s launch, left by an earlier runtime call on this "
                "thread that did not report it: %s",
                kKernelNames[id], hipGetErrorString(pre));
  return RNT_OK;
}

// Bracket one launch with events when profiling is on.
template <class F>
hipError_t prof_launch(const rnt::Tables* t, hipStream_t s, int id, F&& f) {
  rnt::Prof* p = t->prof;
  if (p == nullptr || !p->on || g_capture != nullptr) return f();
  std::lock_guard<std::mutex> g(p->mu);
  hipEvent_t a = prof_event(p), b = prof_event(p);
  bool ok = a && b;
  if (ok) {
    if (const hipError_t r = hipEventRecord(a, s); r != hipSuccess) {
      prof_fail(p, r, "hipEventRecord(profile)");
      ok = false;
    }
  }
  hipError_t e = f();
  if (ok && e == hipSuccess) {
    if (const hipError_t r = hipEventRecord(b, s); r != hipSuccess) {
      prof_fail(p, r, "hipEventRecord(profile)");
      ok = false;
    }
  }
  if (ok && e == hipSuccess) {
    p->pending.push_back({id, a, b});
  } else {
    if (a) p->pool.push_back(a);
    if (b) p->pool.push_back(b);
  }
  return e;
}

// Launch on the context's stream, or (LAUNCH_ON) on an explicit one; with
// profiling on, the launch is bracketed by events on that same stream.
#define LAUNCH(T, ID, EXPR, WHERE)                                           \
  do {                                                                       \
    if (int rc_ = check_pending(ID)) return rc_;                             \
    HIP_TRY(prof_launch((T), (T)->stream, (ID), [&]() { return (EXPR); }), WHERE); \
  } while (0)
#define LAUNCH_ON(T, S, ID, EXPR, WHERE)                                     \
  do {                                                                       \
    if (int rc_ = check_pending(ID)) return rc_;                             \
    HIP_TRY(prof_launch((T), (S), (ID), [&]() { return (EXPR); }), WHERE);   \
  } while (0)



inline rnt::Launch launch_for(const rnt_buf* b) {
  rnt::Launch k;
  k.t = b->ctx->t.get();
  k.L = b->ctx->L;
  k.B = b->n_polys;
  k.s = k.t->stream;
  return k;
}

inline size_t poly_words(const rnt_buf* b) { return b->ctx->L * b->n_polys * b->ctx->t->n; }
inline uint64_t limb_stride(const rnt_buf* b) { return (uint64_t)b->n_polys * b->ctx->t->n; }

int set_device(const rnt_ctx* ctx) {
  HIP_TRY(hipSetDevice(ctx->t->device), "hipSetDevice");
  return RNT_OK;
}

// Device block cache: the data, workspace and staging blocks of freed
// buffers, kept per device for reuse.  A caller that makes fresh buffers
// every step (the limb-sharded pipeline) then reuses the same gigabytes
// instead of a hipMalloc / hipFree per call; that churn made a long ct-mul
// run fall to ~1/15 of its rate after ~30 steps at 128 ciphertexts.
// A freed block carries an event recorded on the stream of its last use.
// The next taker's stream waits on that event (hipStreamWaitEvent), so no
// free makes the host wait for the device; only a block leaving the cache
// (hipFree) waits for its event first.  Idle bytes per device are capped at
// RNT_WS_POOL_MB, by default 1/8 of the device's memory.
struct PoolBlock {
  int device;
  void* p;
  size_t bytes;
  hipEvent_t ev;     // recorded on `s` when the block was freed
  hipStream_t s;
};
std::mutex g_pool_mu;
std::vector<PoolBlock> g_pool;               // oldest first
std::vector<std::pair<int, size_t>> g_pool_bytes;  // idle bytes per device
std::vector<hipEvent_t> g_free_events;       // recycled events

static size_t& pool_bytes_of(int device) {  // g_pool_mu held
  for (auto& e : g_pool_bytes)
    if (e.first == device) return e.second;
  g_pool_bytes.push_back({device, 0});
  return g_pool_bytes.back().second;
}

static size_t pool_cap(int device) {  // g_pool_mu held
  if (const char* e = getenv("RNT_WS_POOL_MB")) {  // read per call: tests set it
    const long mb = atol(e);
    return (size_t)(mb > 0 ? mb : 0) << 20;
  }
  static std::vector<std::pair<int, size_t>> caps;  // default: 1/8 of the device
  for (auto& c : caps)
    if (c.first == device) return c.second;
  size_t free_b = 0, total_b = 0;
  const size_t cap = hipMemGetInfo(&free_b, &total_b) == hipSuccess ? total_b / 8 : ((size_t)8 << 30);
  caps.push_back({device, cap});
  return cap;
}

static void pool_release(const PoolBlock& w) {  // g_pool_mu NOT held
  cleanup(hipSetDevice(w.device), "hipSetDevice(block leaving the cache)");
  if (w.ev) {
    cleanup(hipEventSynchronize(w.ev), "hipEventSynchronize(block leaving the cache)");
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_free_events.push_back(w.ev);
  }
  cleanup(hipFree(w.p), "hipFree(block leaving the cache)");
}

// Smallest idle block on `device` of at least `bytes` (and at most twice
// that, so a small request does not pin a multi-GiB block), made safe to use
// on stream `s`; nullptr if none.
static void* pool_take(int device, size_t bytes, hipStream_t s, size_t* got, bool call_scoped) {
  if (call_scoped && g_capture != nullptr && g_capture->device == device && g_capture->stream == s) {
    OwnedBlock* best = nullptr;
    for (OwnedBlock& o : g_capture->owned)
      if (o.idle && o.bytes >= bytes && o.bytes / 2 <= bytes && (!best || o.bytes < best->bytes)) best = &o;
    if (best) {
      best->idle = false;
      *got = best->bytes;
      return best->p;
    }
  }
  PoolBlock w{};
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    size_t best = g_pool.size();
    for (size_t i = 0; i < g_pool.size(); ++i) {
      const PoolBlock& c = g_pool[i];
      if (c.device == device && c.bytes >= bytes && c.bytes / 2 <= bytes &&
          (best == g_pool.size() || c.bytes < g_pool[best].bytes))
        best = i;
    }
    if (best == g_pool.size()) return nullptr;
    w = g_pool[best];
    pool_bytes_of(device) -= w.bytes;
    g_pool.erase(g_pool.begin() + (long)best);
  }
  if (w.ev) {
    // same stream: stream order already covers the last use; while a graph
    // is being recorded the wait is a host wait (a recording stream cannot
    // wait on an event from outside the recording)
    if (w.s != s) {
      const hipError_t we = g_capture != nullptr ? hipErrorStreamCaptureUnsupported : hipStreamWaitEvent(s, w.ev, 0);
      if (we != hipSuccess) {
        if (g_capture == nullptr) (void)hipGetLastError();  // handled: a host wait instead
        cleanup(hipEventSynchronize(w.ev), "hipEventSynchronize(block from the cache)");
      }
    }
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_free_events.push_back(w.ev);
  }
  *got = w.bytes;
  return w.p;
}

// Hand a block whose last use was queued on stream `s` to the cache; the
// oldest idle blocks of the device leave it while it is over its cap.
static void pool_give(int device, void* p, size_t bytes, hipStream_t s) {
  if (!p) return;
  if (g_capture != nullptr && g_capture->device == device && g_capture->stream == s) {
    // the recorded graph keeps using the block
    for (OwnedBlock& o : g_capture->owned)
      if (o.p == p) {
        o.idle = true;
        return;
      }
    g_capture->owned.push_back({p, bytes, true});
    return;
  }
  hipEvent_t ev = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (!g_free_events.empty()) {
      ev = g_free_events.back();
      g_free_events.pop_back();
    }
  }
  if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) ev = nullptr;
  if (!ev) (void)hipGetLastError();  // handled: drain instead
  if (ev && hipEventRecord(ev, s) != hipSuccess) {
    (void)hipGetLastError();  // handled: drain instead
    cleanup(hipStreamSynchronize(s), "hipStreamSynchronize(block handed to the cache)");
    cleanup(hipEventDestroy(ev), "hipEventDestroy(block handed to the cache)");
    ev = nullptr;
  } else if (!ev) {
    cleanup(hipStreamSynchronize(s), "hipStreamSynchronize(block handed to the cache)");
  }
  std::vector<PoolBlock> drop;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_pool.push_back({device, p, bytes, ev, s});
    size_t& idle = pool_bytes_of(device);
    idle += bytes;
    const size_t cap = pool_cap(device);
    for (size_t i = 0; idle > cap && i < g_pool.size();) {
      if (g_pool[i].device == device) {
        drop.push_back(g_pool[i]);
        idle -= g_pool[i].bytes;
        g_pool.erase(g_pool.begin() + (long)i);
      } else {
        ++i;
      }
    }
  }
  for (const PoolBlock& w : drop) pool_release(w);
  if (!drop.empty()) cleanup(hipSetDevice(device), "hipSetDevice(after the cache's release)");
}

// Free every idle block of `device` (-1: of every device).
static size_t pool_drain(int device) {
  std::vector<PoolBlock> drop;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (size_t i = 0; i < g_pool.size();) {
      if (device < 0 || g_pool[i].device == device) {
        drop.push_back(g_pool[i]);
        pool_bytes_of(g_pool[i].device) -= g_pool[i].bytes;
        g_pool.erase(g_pool.begin() + (long)i);
      } else {
        ++i;
      }
    }
  }
  size_t freed = 0;
  for (const PoolBlock& w : drop) {
    freed += w.bytes;
    pool_release(w);
  }
  return freed;
}

// A device block of at least `bytes` for work on stream `s`: from the cache,
// else hipMalloc (after emptying the device's cache if that fails).
static hipError_t pool_malloc(int device, size_t bytes, hipStream_t s, void** p, size_t* got,
                              bool call_scoped = false) {
  if ((*p = pool_take(device, bytes, s, got, call_scoped))) return hipSuccess;
  hipError_t e = hipMalloc(p, bytes);
  if (e == hipErrorOutOfMemory) {
    (void)hipGetLastError();
    if (pool_drain(device) > 0) {
      cleanup(hipSetDevice(device), "hipSetDevice(after draining the cache)");
      e = hipMalloc(p, bytes);
    }
  }
  if (e != hipSuccess) {
    *p = nullptr;
    return e;
  }
  *got = bytes;
  return hipSuccess;
}

// Grow the buffer's private workspace to at least `bytes`.
int ensure_ws(rnt_buf* b, size_t bytes) {
  if (b->ws_bytes >= bytes) return RNT_OK;
  const int dev = b->ctx->t->device;
  hipStream_t s = b->ctx->t->stream;
  if (b->ws) {
    pool_give(dev, b->ws, b->ws_bytes, s);  // the stream may still be using it
    b->ws = nullptr;
    b->ws_bytes = 0;
  }
  size_t got = 0;
  if (hipError_t e = pool_malloc(dev, bytes, s, &b->ws, &got); e != hipSuccess)
    return hip_fail(e, "hipMalloc(workspace)");
  b->ws_bytes = got;
  return RNT_OK;
}

// A call-scoped device workspace from the block cache: taken when an op
// starts and handed back when the call returns, behind an event on the op's
// stream (no host wait), so the next op -- on any buffer -- reuses the same
// block.  Key-switch scratch (gigabytes per chunk) lives here rather than
// with an output buffer: a caller that makes a fresh output per chunk (the
// limb-sharded pipeline) would otherwise hold one scratch per live output.
struct CallWs {
  int dev;
  hipStream_t s;
  void* p = nullptr;
  size_t bytes = 0;
  explicit CallWs(const rnt_buf* b) : dev(b->ctx->t->device), s(b->ctx->t->stream) {}
  CallWs(const CallWs&) = delete;
  CallWs& operator=(const CallWs&) = delete;
  int get(size_t need) {
    size_t got = 0;
    if (hipError_t e = pool_malloc(dev, need, s, &p, &got, true); e != hipSuccess)
      return hip_fail(e, "hipMalloc(workspace)");
    bytes = got;
    return RNT_OK;
  }
  ~CallWs() {
    if (p) pool_give(dev, p, bytes, s);
  }
};

int ensure_stage(rnt_buf* b, size_t bytes) {
  if (b->stage_bytes >= bytes) return RNT_OK;
  const int dev = b->ctx->t->device;
  hipStream_t s = b->ctx->t->stream;
  if (b->stage) {
    pool_give(dev, b->stage, b->stage_bytes, s);
    b->stage = nullptr;
    b->stage_bytes = 0;
  }
  size_t got = 0;
  if (hipError_t e = pool_malloc(dev, bytes, s, &b->stage, &got); e != hipSuccess)
    return hip_fail(e, "hipMalloc(stage)");
  b->stage_bytes = got;
  return RNT_OK;
}

// Staging for uploads/downloads stays with its buffer, except very large
// ones (a 256-poly batch at N=2^16, L=16 stages 2 GiB of u64), which go back
// to the cache.
void trim_stage(rnt_buf* b) {
  if (b->stage_bytes > ((size_t)256 << 20)) {
    pool_give(b->ctx->t->device, b->stage, b->stage_bytes, b->ctx->t->stream);
    b->stage = nullptr;
    b->stage_bytes = 0;
  }
}

int check_buf(const rnt_buf* b, const char* name) {
  if (b == nullptr || b->ctx == nullptr) return fail(RNT_ERR_BAD_ARGUMENT, "%s: null buffer", name);
  return RNT_OK;
}

// Same basis (Arc::ptr_eq on the basis in the reference) and batch size.
int check_same(const rnt_buf* a, const rnt_buf* b, const char* what) {
  if (a->ctx != b->ctx)
    return fail(RNT_ERR_BASIS_MISMATCH, "%s: operands belong to different bases", what);
  if (a->n_polys != b->n_polys)
    return fail(RNT_ERR_BAD_ARGUMENT, "%s: batch sizes differ (%zu vs %zu)", what, a->n_polys,
                b->n_polys);
  return RNT_OK;
}

// The MFMA transforms (rnt_mfma.hip) for this context: N = 2^16 on a u32
// basis (unless RNT_PLANE=0).  Their tables are built with the context
// (rnt_ctx_create), so no op -- none recorded into a graph either -- ever
// builds them, and a context whose build failed does not exist.
bool use_mf(const rnt::Launch& k) { return rnt::mf_supported(k.t) && k.t->mf != nullptr; }

// Inverse-transform src (NTT domain) into dst (same layout): dst may equal src.
int to_coeff_into(const rnt_buf* src, void* dst) {
  rnt::Launch k = launch_for(src);
  const uint64_t ls = limb_stride(src);
  if (dst != src->data)
    HIP_TRY(hipMemcpyAsync(dst, src->data, poly_words(src) * word_bytes(k.t),
                           hipMemcpyDeviceToDevice, k.s),
            "hipMemcpyAsync");
  if (use_mf(k)) {
    LAUNCH(k.t, rnt::K_MF_NTT_INV, rnt::launch_mf_ntt(k, 1, dst, ls), "MFMA inverse transform");
    return RNT_OK;
  }
  if (rnt::whole_ok(k.t, 1)) {
    LAUNCH(k.t, rnt::K_WHOLE_INV, rnt::launch_whole(k, 1, dst, dst, nullptr, ls), "whole-plane inverse");
    return RNT_OK;
  }
  LAUNCH(k.t, rnt::K_ROW_INV, rnt::launch_row(k, 1, dst, nullptr, ls), "row inverse");
  LAUNCH(k.t, rnt::K_COL_INV, rnt::launch_col_inv(k, dst, ls, dst, ls, 0, nullptr), "column inverse");
  return RNT_OK;
}

}  // namespace

rnt::Tables::~Tables() {
  cleanup(hipSetDevice(device), "hipSetDevice(context teardown)");
  if (stream && stream != own_stream)  // a caller's stream
    cleanup(hipStreamSynchronize(stream), "hipStreamSynchronize(context teardown)");
  if (own_stream) {
    cleanup(hipStreamSynchronize(own_stream), "hipStreamSynchronize(context teardown)");
    cleanup(hipStreamDestroy(own_stream), "hipStreamDestroy(context teardown)");
  }
  for (auto& e : resc_ext) cleanup(hipFree(e.second), "hipFree(context tables)");
  for (auto& e : crt_cache) cleanup(hipFree(e.second.dev), "hipFree(context tables)");
  for (void* p : {tw_fwd, tw_inv, sfft_tw, lconst, resc, resc_p, mf})
    cleanup(hipFree(p), "hipFree(context tables)");
  if (prof) {
    for (auto& r : prof->pending) {
      cleanup(hipEventDestroy(r.a), "hipEventDestroy(profile)");
      cleanup(hipEventDestroy(r.b), "hipEventDestroy(profile)");
    }
    for (hipEvent_t e : prof->pool) cleanup(hipEventDestroy(e), "hipEventDestroy(profile)");
    delete prof;
  }
}

static long env_long(const char* name, long dflt);

// ---------------------------------------------------------------------------
// diagnostics
// ---------------------------------------------------------------------------
extern "C" int rnt_abi_version(void) { return RNT_ABI_VERSION; }
extern "C" int rnt_last_error_detail(uint64_t fields[2]) {
  if (fields) {
    fields[0] = g_last_detail.a;
    fields[1] = g_last_detail.b;
  }
  return g_last_detail.status;
}

extern "C" const char* rnt_last_error(void) { return g_last_error.c_str(); }
extern "C" const char* rnt_status_string(int s) {
  switch (s) {
    case RNT_OK: return "ok";
    case RNT_ERR_INVALID_DEGREE: return "InvalidDegree";
    case RNT_ERR_EMPTY_BASIS: return "EmptyBasis";
    case RNT_ERR_NON_NTT_FRIENDLY: return "NonNttFriendlyModulus";
    case RNT_ERR_INVALID_MOD_DROP: return "InvalidModDrop";
    case RNT_ERR_CHANNEL_COUNT: return "ChannelCountMismatch";
    case RNT_ERR_NON_REDUCED: return "NonReducedCoefficient";
    case RNT_ERR_DOMAIN_MISMATCH: return "DomainMismatch";
    case RNT_ERR_BASIS_MISMATCH: return "BasisMismatch";
    case RNT_ERR_DEVICE: return "DeviceError";
    case RNT_ERR_OUT_OF_MEMORY: return "OutOfMemory";
    case RNT_ERR_BAD_ARGUMENT: return "BadArgument";
    case RNT_ERR_UNSUPPORTED: return "Unsupported";
    default: return "unknown";
  }
}

// ---------------------------------------------------------------------------
// host-side number theory
// ---------------------------------------------------------------------------
extern "C" int rnt_is_ntt_friendly_prime(uint64_t p, uint64_t degree, int* out) {
  if (!out) return fail(RNT_ERR_BAD_ARGUMENT, "null out");
  if (degree == 0 || degree > UINT64_MAX / 2)
    return fail(RNT_ERR_BAD_ARGUMENT, "is_ntt_friendly_prime: degree must be in [1, 2^63)");
  *out = rnt::host::is_ntt_friendly(p, degree) ? 1 : 0;
  return RNT_OK;
}

extern "C" int rnt_generate_primes(uint32_t bit_size, size_t count, uint64_t degree,
                                   uint64_t* out) {
  if (!out && count) return fail(RNT_ERR_BAD_ARGUMENT, "null out");
  if (rnt::host::generate_primes(bit_size, count, degree, out) != 0)
    return fail(RNT_ERR_BAD_ARGUMENT,
                "Unable to find %zu NTT primes with %u-bit ceiling for degree %" PRIu64, count,
                bit_size, degree);
  return RNT_OK;
}

extern "C" int rnt_find_psi(uint64_t modulus, uint64_t degree, uint64_t* psi) {
  if (!psi) return fail(RNT_ERR_BAD_ARGUMENT, "null out");
  if (degree == 0 || (degree & (degree - 1)))
    return fail_fields(RNT_ERR_INVALID_DEGREE, degree, 0, "ring degree must be a power of two, got %" PRIu64,
                       degree);
  if (!rnt::host::is_ntt_friendly(modulus, degree))
    return fail_fields(RNT_ERR_NON_NTT_FRIENDLY, modulus, degree,
                       "modulus %" PRIu64 " is not NTT-friendly for degree %" PRIu64,
                modulus, degree);
  *psi = rnt::host::find_psi(modulus, degree);
  return RNT_OK;
}

// ---------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------
namespace {

template <class W>
int build_tables(rnt::Tables* t) {
  using namespace rnt::host;
  const size_t n = t->n, L = t->L;
  const unsigned wbits = sizeof(W) * 8;
  std::vector<rnt::Tw<W>> tw(L * n), itw(L * n);
  std::vector<rnt::LimbConst<W>> lc(L);
  std::vector<W> resc(L * L, 0), rescp(L * L, 0);
  std::vector<uint64_t> pw(n), ipw(n);
  for (size_t l = 0; l < L; ++l) {
    const uint64_t q = t->moduli[l];
    const uint64_t psi = find_psi(q, n);
    if (psi == 0)
      return fail_fields(RNT_ERR_NON_NTT_FRIENDLY, q, n, "no primitive 2N-th root mod %" PRIu64, q);
    t->psi.push_back(psi);
    const uint64_t psi_inv = invmod(psi, q);
    uint64_t a = 1, b = 1;
    for (size_t j = 0; j < n; ++j) {
      pw[j] = a;
      ipw[j] = b;
      a = mulmod(a, psi, q);
      b = mulmod(b, psi_inv, q);
    }
    rnt::Tw<W>* T = tw.data() + l * n;
    rnt::Tw<W>* I = itw.data() + l * n;
    T[0] = {(W)1, (W)shoup_companion(1, q, wbits)};
    I[0] = T[0];
    for (size_t g = 1; g < n; ++g) {
      const uint64_t e = brv(g, t->log_n);
      T[g] = {(W)pw[e], (W)shoup_companion(pw[e], q, wbits)};
      I[g] = {(W)ipw[e], (W)shoup_companion(ipw[e], q, wbits)};
    }
    rnt::LimbConst<W>& c = lc[l];
    c.q = (W)q;
    c.qinv = (W)neg_free_qinv(q, wbits);
    c.one_p = (W)shoup_companion(1, q, wbits);
    const uint64_t r = (uint64_t)((((u128)1) << wbits) % q);  // 2^w mod q
    c.rmod = (W)r;
    c.rmod_p = (W)shoup_companion(r, q, wbits);
    const uint64_t ninv = invmod(n % q, q);
    const uint64_t w1 = n > 1 ? (uint64_t)I[1].w : 1;
    c.c1 = (W)ninv;
    c.c1_p = (W)shoup_companion(ninv, q, wbits);
    c.c2 = (W)mulmod(w1, ninv, q);
    c.c2_p = (W)shoup_companion(c.c2, q, wbits);
    const uint64_t ninvr = mulmod(ninv, r, q);
    c.c1r = (W)ninvr;
    c.c1r_p = (W)shoup_companion(ninvr, q, wbits);
    c.c2r = (W)mulmod(w1, ninvr, q);
    c.c2r_p = (W)shoup_companion(c.c2r, q, wbits);
    const uint64_t ninvrt = mulmod(ninvr, 4 % q, q);
    c.c1t = (W)ninvrt;
    c.c1t_p = (W)shoup_companion(ninvrt, q, wbits);
    c.c2t = (W)mulmod(w1, ninvrt, q);
    c.c2t_p = (W)shoup_companion(c.c2t, q, wbits);
    for (size_t i = 0; i < l; ++i) {
      const uint64_t qi = t->moduli[i];
      const uint64_t inv = invmod(q % qi, qi);
      if (inv == 0)
        return fail(RNT_ERR_BAD_ARGUMENT, "moduli %" PRIu64 " and %" PRIu64 " are not coprime", q, qi);
      resc[l * L + i] = (W)inv;
      rescp[l * L + i] = (W)shoup_companion(inv, qi, wbits);
    }
  }
  const size_t tb = L * n * sizeof(rnt::Tw<W>);
  HIP_TRY(hipMalloc(&t->tw_fwd, tb), "hipMalloc(tables)");
  HIP_TRY(hipMalloc(&t->tw_inv, tb), "hipMalloc(tables)");
  HIP_TRY(hipMalloc(&t->lconst, L * sizeof(rnt::LimbConst<W>)), "hipMalloc(tables)");
  HIP_TRY(hipMalloc(&t->resc, L * L * sizeof(W)), "hipMalloc(tables)");
  HIP_TRY(hipMalloc(&t->resc_p, L * L * sizeof(W)), "hipMalloc(tables)");
  HIP_TRY(hipMemcpy(t->tw_fwd, tw.data(), tb, hipMemcpyHostToDevice), "hipMemcpy");
  HIP_TRY(hipMemcpy(t->tw_inv, itw.data(), tb, hipMemcpyHostToDevice), "hipMemcpy");
  HIP_TRY(hipMemcpy(t->lconst, lc.data(), L * sizeof(rnt::LimbConst<W>), hipMemcpyHostToDevice),
          "hipMemcpy");
  HIP_TRY(hipMemcpy(t->resc, resc.data(), L * L * sizeof(W), hipMemcpyHostToDevice), "hipMemcpy");
  HIP_TRY(hipMemcpy(t->resc_p, rescp.data(), L * L * sizeof(W), hipMemcpyHostToDevice),
          "hipMemcpy");
  return RNT_OK;
}

}  // namespace

extern "C" int rnt_ctx_create(uint32_t log_n, const uint64_t* moduli, size_t count, int device,
                              rnt_ctx** out) {
  if (!out) return fail(RNT_ERR_BAD_ARGUMENT, "null out");
  *out = nullptr;
  // RnsBasis::new order (basis.rs:97-106): empty basis first, then each
  // NttTable::new (degree check, NTT-friendliness).
  if (count == 0) return fail(RNT_ERR_EMPTY_BASIS, "RNS basis must contain at least one modulus");
  if (!moduli) return fail(RNT_ERR_BAD_ARGUMENT, "null moduli");
  // log_n is the exponent of a power of two, so the reference's
  // InvalidDegree (basis.rs:22-24, "not a power of two") cannot arise here;
  // the Python/C++ mirrors raise it before calling.
  if (log_n >= 63) return fail(RNT_ERR_BAD_ARGUMENT, "log_n %u out of range", log_n);
  const uint64_t n = 1ull << log_n;
  bool wide = false, lazy30 = true, lazy62 = true;
  for (size_t i = 0; i < count; ++i) {
    if (!rnt::host::is_ntt_friendly(moduli[i], n))
      return fail_fields(RNT_ERR_NON_NTT_FRIENDLY, moduli[i], n,
                         "modulus %" PRIu64 " is not NTT-friendly for degree %" PRIu64, moduli[i], n);
    if (moduli[i] >= (1ull << 63))
      return fail(RNT_ERR_BAD_ARGUMENT,
                  "modulus %" PRIu64 " >= 2^63 (the reference's add_mod overflows)", moduli[i]);
    if (moduli[i] >= (1ull << 31)) wide = true;
    if (moduli[i] >= (1ull << 30)) lazy30 = false;
    if (moduli[i] >= (1ull << 62)) lazy62 = false;
  }
  // a valid basis the reference would accept, beyond this backend's tables
  // and grids: its own capacity status, not the reference's InvalidDegree
  if (log_n > (uint32_t)rnt::kMaxLogN)
    return fail_fields(RNT_ERR_UNSUPPORTED, n, 1ull << rnt::kMaxLogN,
                       "ring degree 2^%u exceeds this backend's maximum 2^%d (Unsupported, not "
                       "InvalidDegree: the degree is valid for the reference)",
                       log_n, rnt::kMaxLogN);
  try {
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
    if (device < 0 || device >= ndev)
      return fail(RNT_ERR_BAD_ARGUMENT, "device %d out of range (%d devices)", device, ndev);
    HIP_TRY(hipSetDevice(device), "hipSetDevice");
    auto t = std::make_shared<rnt::Tables>();
    t->device = device;
    t->wide = wide ? 1 : 0;
    // RNT_LAZY30=0 keeps the canonical product path for 30-bit bases (A/B)
    t->lazy30 = !wide && lazy30 && env_long("RNT_LAZY30", 1) != 0;
    // the same Harvey-lazy product path for u64 bases of primes < 2^62 (the
    // reference's 40/61/62-bit tests); RNT_LAZY62=0 keeps the canonical one
    t->lazy62 = wide && lazy62 && env_long("RNT_LAZY62", 1) != 0;
    // the ct-mul's key-switch takes its diagonal (source limb i of target
    // limb i) from the tensor's exact d2^ instead of transforming it;
    // RNT_KS_DIAG=0 transforms every (i, j) (A/B)
    t->ks_diag = env_long("RNT_KS_DIAG", 1) != 0;
    t->rot_fuse = (int)env_long("RNT_ROT_FUSE", 1);
    // the whole-plane product and MFMA transforms are the default where they
    // apply (N = 2^16, u32); RNT_PLANE=0 keeps the four-step kernels
    t->plane = env_long("RNT_PLANE", 1) != 0 ? 1 : 0;
    // the product on the matrix-core transforms (k_mf_mul) where they apply;
    // RNT_MF_MUL=0 keeps the VALU whole-plane product (k_plane_fused_slots)
    t->mf_mul = env_long("RNT_MF_MUL", 1) != 0 ? 1 : 0;
    {
      const long jg = env_long("RNT_DEC_JG", 0);  // A/B knob: 0 = auto, else 1..1024
      t->dec_jg = (uint32_t)(jg < 0 ? 0 : jg > 1024 ? 1024 : jg);
      // key-switch scratch cap (S = [L][L][Bc][N] words per chunk), MiB.
      // 16 GiB: 256-ct chunks at config 4 (N = 2^16, L = 16) ran the fused
      // ct-mul 2.5% faster than 64-ct ones (4 GiB), the tensor and rows
      // kernels' last-round tails amortised over 4x the grid; 32 GiB chunks
      // fell off the workspace pool (profiles/r06/ab_ks_chunk.txt)
      const long mb = env_long("RNT_KS_WS_MB", 16384);
      t->ks_ws_bytes = (size_t)(mb > 0 ? mb : 16384) << 20;
    }
    t->log_n = log_n;
    t->n = (size_t)n;
    t->L = count;
    t->moduli.assign(moduli, moduli + count);
    int rc = wide ? build_tables<uint64_t>(t.get()) : build_tables<uint32_t>(t.get());
    if (rc != RNT_OK) return rc;
    if (rnt::mf_supported(t.get())) {
      std::string err;
      if (const int m = rnt::mf_build(t.get(), &err); m != 0) {
        (void)hipGetLastError();  // reported here
        return fail(m == -3 ? RNT_ERR_OUT_OF_MEMORY : RNT_ERR_DEVICE, "%s", err.c_str());
      }
    }
    HIP_TRY(hipStreamCreateWithFlags(&t->own_stream, hipStreamNonBlocking), "hipStreamCreate");
    t->stream = t->own_stream;
    rnt_ctx* c = new rnt_ctx;
    c->t = std::move(t);
    c->L = count;
    *out = c;
    return RNT_OK;
  } catch (const std::bad_alloc&) {
    return fail(RNT_ERR_OUT_OF_MEMORY, "host allocation failed");
  } catch (...) {
    return fail(RNT_ERR_DEVICE, "unexpected exception in rnt_ctx_create");
  }
}

static void ctx_release(const rnt_ctx* ctx) {
  if (ctx && const_cast<rnt_ctx*>(ctx)->refs.fetch_sub(1) == 1) delete ctx;
}
static void ctx_retain(const rnt_ctx* ctx) { const_cast<rnt_ctx*>(ctx)->refs.fetch_add(1); }

extern "C" int rnt_ctx_destroy(rnt_ctx* ctx) {
  OwnCleanup own;
  ctx_release(ctx);  // freed once its last buffer is freed too
  return own.finish();
}

extern "C" int rnt_ctx_drop_last(const rnt_ctx* ctx, size_t drop_count, rnt_ctx** out) {
  if (!ctx || !out) return fail(RNT_ERR_BAD_ARGUMENT, "null argument");
  *out = nullptr;
  if (drop_count >= ctx->L)
    return fail_fields(RNT_ERR_INVALID_MOD_DROP, drop_count, ctx->L,
                       "invalid mod-drop count %zu for %zu channels", drop_count, ctx->L);
  try {
    rnt_ctx* c = new rnt_ctx;
    c->t = ctx->t;
    c->L = ctx->L - drop_count;
    *out = c;
  } catch (...) {
    return fail(RNT_ERR_OUT_OF_MEMORY, "host allocation failed");
  }
  return RNT_OK;
}

extern "C" int rnt_ctx_degree(const rnt_ctx* ctx, size_t* n) {
  if (!ctx || !n) return fail(RNT_ERR_BAD_ARGUMENT, "null argument");
  *n = ctx->t->n;
  return RNT_OK;
}
extern "C" int rnt_ctx_channel_count(const rnt_ctx* ctx, size_t* count) {
  if (!ctx || !count) return fail(RNT_ERR_BAD_ARGUMENT, "null argument");
  *count = ctx->L;
  return RNT_OK;
}
extern "C" int rnt_ctx_moduli(const rnt_ctx* ctx, uint64_t* out) {
  if (!ctx || !out) return fail(RNT_ERR_BAD_ARGUMENT, "null argument");
  std::copy(ctx->t->moduli.begin(), ctx->t->moduli.begin() + ctx->L, out);
  return RNT_OK;
}
extern "C" int rnt_ctx_total_bits(const rnt_ctx* ctx, uint32_t* bits) {
  if (!ctx || !bits) return fail(RNT_ERR_BAD_ARGUMENT, "null argument");
  uint32_t s = 0;
  for (size_t i = 0; i < ctx->L; ++i) s += 63u - (uint32_t)__builtin_clzll(ctx->t->moduli[i]);
  *bits = s;
  return RNT_OK;
}
extern "C" int rnt_ctx_psi(const rnt_ctx* ctx, size_t limb, uint64_t* psi) {
  if (!ctx || !psi) return fail(RNT_ERR_BAD_ARGUMENT, "null argument");
  if (limb >= ctx->L) return fail(RNT_ERR_BAD_ARGUMENT, "limb %zu out of range", limb);
  *psi = ctx->t->psi[limb];
  return RNT_OK;
}
extern "C" int rnt_ctx_stream(const rnt_ctx* ctx, void** stream) {
  if (!ctx || !stream) return fail(RNT_ERR_BAD_ARGUMENT, "null argument");
  *stream = (void*)ctx->t->stream;
  return RNT_OK;
}
// Later ops go to `stream` (NULL: the context's own) after everything queued
// so far: the new stream waits on an event recorded on the old one.
extern "C" int rnt_ctx_set_stream(const rnt_ctx* ctx, void* stream) {
  if (!ctx) return fail(RNT_ERR_BAD_ARGUMENT, "null ctx");
  if (int rc = set_device(ctx)) return rc;
  rnt::Tables* t = ctx->t.get();
  hipStream_t next = stream ? (hipStream_t)stream : t->own_stream;
  if (next == t->stream) return RNT_OK;
  if (stream) {
    hipDevice_t dev = -1;
    HIP_TRY(hipStreamGetDevice(next, &dev), "hipStreamGetDevice");
    if (dev != t->device)
      return fail(RNT_ERR_BAD_ARGUMENT, "stream is on device %d, the context on device %d", (int)dev,
                  t->device);
  }
  hipEvent_t ev;
  HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
  hipError_t e = hipEventRecord(ev, t->stream);
  if (e == hipSuccess) e = hipStreamWaitEvent(next, ev, 0);
  cleanup(hipEventDestroy(ev), "hipEventDestroy(rnt_ctx_set_stream)");  // released once it completes
  if (e != hipSuccess) return hip_fail(e, "rnt_ctx_set_stream");
  t->stream = next;
  return RNT_OK;
}

// ---------------------------------------------------------------------------
// captured op sequences (hipGraph)
// ---------------------------------------------------------------------------
// A recorded graph owns the distinct workspace blocks its ops took (on
// `device`); they go back to the cache when it is destroyed, behind an event
// on `last` -- the stream the latest replay was queued on.  A replay on a
// new stream (after rnt_ctx_set_stream) is first ordered after the previous
// replays, so `last` covers every replay.
// `done`: recorded after each replay, so the next replay (on whatever
// stream the context uses by then) and the blocks' return to the cache wait
// for it -- no stream handle outlives its use here.
struct rnt_graph {
  std::shared_ptr<rnt::Tables> t;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  std::vector<OwnedBlock> owned;
  int device = 0;
  hipEvent_t done = nullptr;
  bool replayed = false;
};

extern "C" int rnt_capture_begin(const rnt_ctx* ctx) {
  if (!ctx) return fail(RNT_ERR_BAD_ARGUMENT, "null ctx");
  if (g_capture != nullptr) return fail(RNT_ERR_BAD_ARGUMENT, "rnt_capture_begin: already recording on this thread");
  if (int rc = set_device(ctx)) return rc;
  Capture* c = nullptr;
  try {
    c = new Capture;
  } catch (...) {
    return fail(RNT_ERR_OUT_OF_MEMORY, "host allocation failed");
  }
  c->stream = ctx->t->stream;
  c->device = ctx->t->device;
  // relaxed: the ops' own host-side calls (none synchronising once warm)
  // are not checked against the recording
  if (hipError_t e = hipStreamBeginCapture(c->stream, hipStreamCaptureModeRelaxed); e != hipSuccess) {
    delete c;
    return hip_fail(e, "hipStreamBeginCapture");
  }
  g_capture = c;
  return RNT_OK;
}

extern "C" int rnt_capture_end(const rnt_ctx* ctx, rnt_graph** out) {
  if (!ctx || !out) return fail(RNT_ERR_BAD_ARGUMENT, "null argument");
  *out = nullptr;
  Capture* c = g_capture;
  if (c == nullptr || c->stream != ctx->t->stream)
    return fail(RNT_ERR_BAD_ARGUMENT, "rnt_capture_end: no recording on this context's stream");
  g_capture = nullptr;
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(c->stream, &g);
  rnt_graph* r = nullptr;
  if (e == hipSuccess) {
    try {
      r = new rnt_graph;
    } catch (...) {
      e = hipErrorOutOfMemory;
    }
  }
  if (r != nullptr) {
    r->t = ctx->t;
    r->graph = g;
    r->owned = std::move(c->owned);
    r->device = c->device;
    e = hipEventCreateWithFlags(&r->done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipGraphInstantiate(&r->exec, g, nullptr, nullptr, 0);
  }
  if (e != hipSuccess) {
    const int dev = c->device;
    const hipStream_t st = c->stream;
    std::vector<OwnedBlock> owned = r ? std::move(r->owned) : std::move(c->owned);
    if (g) cleanup(hipGraphDestroy(g), "hipGraphDestroy(failed capture)");
    if (r && r->done) cleanup(hipEventDestroy(r->done), "hipEventDestroy(failed capture)");
    delete r;
    delete c;
    for (auto& b : owned) pool_give(dev, b.p, b.bytes, st);
    return hip_fail(e, "rnt_capture_end");
  }
  delete c;
  *out = r;
  return RNT_OK;
}

extern "C" int rnt_graph_launch(rnt_graph* g) {
  if (!g) return fail(RNT_ERR_BAD_ARGUMENT, "null graph");
  if (g_capture != nullptr) return fail(RNT_ERR_BAD_ARGUMENT, "rnt_graph_launch while recording");
  HIP_TRY(hipSetDevice(g->device), "hipSetDevice");
  hipStream_t s = g->t->stream;
  if (int rc = take_deferred()) return rc;
  // after the previous replay, wherever it was queued (same stream: free)
  if (g->replayed) HIP_TRY(hipStreamWaitEvent(s, g->done, 0), "hipStreamWaitEvent");
  HIP_TRY(hipGraphLaunch(g->exec, s), "hipGraphLaunch");
  HIP_TRY(hipEventRecord(g->done, s), "hipEventRecord");
  g->replayed = true;
  return RNT_OK;
}

extern "C" int rnt_graph_destroy(rnt_graph* g) {
  if (!g) return RNT_OK;
  OwnCleanup own;
  cleanup(hipSetDevice(g->device), "hipSetDevice(rnt_graph_destroy)");
  // a replay may still be running: the blocks go back to the cache behind
  // the context's current stream, made to wait for the last replay first
  hipStream_t s = g->t->stream;
  if (g->replayed) cleanup(hipStreamWaitEvent(s, g->done, 0), "hipStreamWaitEvent(rnt_graph_destroy)");
  for (auto& b : g->owned) pool_give(g->device, b.p, b.bytes, s);
  if (g->exec) cleanup(hipGraphExecDestroy(g->exec), "hipGraphExecDestroy");
  if (g->graph) cleanup(hipGraphDestroy(g->graph), "hipGraphDestroy");
  if (g->done) cleanup(hipEventDestroy(g->done), "hipEventDestroy(rnt_graph_destroy)");
  delete g;
  return own.finish();
}

extern "C" int rnt_graph_workspace(const rnt_graph* g, size_t* blocks, size_t* bytes) {
  if (!g || !blocks || !bytes) return fail(RNT_ERR_BAD_ARGUMENT, "null argument");
  *blocks = g->owned.size();
  *bytes = 0;
  for (const OwnedBlock& b : g->owned) *bytes += b.bytes;
  return RNT_OK;
}

extern "C" int rnt_sync(const rnt_ctx* ctx) {
  if (!ctx) return fail(RNT_ERR_BAD_ARGUMENT, "null ctx");
  if (int rc = set_device(ctx)) return rc;
  HIP_TRY(hipStreamSynchronize(ctx->t->stream), "hipStreamSynchronize");
  return RNT_OK;
}

// ---------------------------------------------------------------------------
// buffers
// ---------------------------------------------------------------------------
static int buf_alloc(const rnt_ctx* ctx, size_t n_polys, rnt_buf** out, bool zero);

extern "C" int rnt_buf_alloc(const rnt_ctx* ctx, size_t n_polys, rnt_buf** out) {
  return buf_alloc(ctx, n_polys, out, true);
}

// An op's output buffer: the op overwrites every word, so the zero fill
// (a fill kernel of the whole buffer on the stream: 33 us per 16 MiB, two
// per ct-mul chunk for the tensor's d0^/d1^) is skipped.
extern "C" int rnt_buf_alloc_uninit(const rnt_ctx* ctx, size_t n_polys, rnt_buf** out) {
  return buf_alloc(ctx, n_polys, out, false);
}

static int buf_alloc(const rnt_ctx* ctx, size_t n_polys, rnt_buf** out, bool zero) {
  if (!ctx || !out) return fail(RNT_ERR_BAD_ARGUMENT, "null argument");
  *out = nullptr;
  if (n_polys == 0) return fail(RNT_ERR_BAD_ARGUMENT, "n_polys must be positive");
  if (int rc = set_device(ctx)) return rc;
  rnt_buf* b = nullptr;
  try {
    b = new rnt_buf;
  } catch (...) {
    return fail(RNT_ERR_OUT_OF_MEMORY, "host allocation failed");
  }
  b->ctx = ctx;
  const_cast<rnt_ctx*>(ctx)->refs.fetch_add(1);
  b->n_polys = n_polys;
  const size_t bytes = poly_words(b) * word_bytes(ctx->t.get());
  hipStream_t s = ctx->t->stream;
  hipError_t e = pool_malloc(ctx->t->device, bytes, s, &b->data, &b->data_bytes);
  if (e != hipSuccess) {
    ctx_release(ctx);
    delete b;
    return hip_fail(e, "hipMalloc(buffer)");
  }
  // zero (RnsPoly::zero), queued on the context stream like every op
  if (zero) e = hipMemsetAsync(b->data, 0, bytes, s);
  if (e != hipSuccess) {
    pool_give(ctx->t->device, b->data, b->data_bytes, s);
    ctx_release(ctx);
    delete b;
    return hip_fail(e, "hipMemset(buffer)");
  }
  *out = b;
  return RNT_OK;
}

// No host wait: the blocks go to the device cache with an event on the
// context stream, behind every op queued on this buffer.
extern "C" int rnt_buf_free(rnt_buf* b) {
  if (!b) return RNT_OK;
  OwnCleanup own;
  if (b->ctx) {
    const int dev = b->ctx->t->device;
    hipStream_t s = b->ctx->t->stream;
    cleanup(hipSetDevice(dev), "hipSetDevice(rnt_buf_free)");
    if (b->owns) pool_give(dev, b->data, b->data_bytes, s);
    pool_give(dev, b->ws, b->ws_bytes, s);
    pool_give(dev, b->stage, b->stage_bytes, s);
  }
  ctx_release(b->ctx);
  delete b;
  return own.finish();
}

extern "C" int rnt_debug_defer(int hip_error) {
  if (hip_error == 0) return fail(RNT_ERR_BAD_ARGUMENT, "rnt_debug_defer: hip_error must be nonzero");
  cleanup(static_cast<hipError_t>(hip_error), "rnt_debug_defer");
  return RNT_OK;
}

extern "C" int rnt_pool_trim(int device, size_t* freed_bytes) {
  OwnCleanup own;
  const size_t f = pool_drain(device);
  if (freed_bytes) *freed_bytes = f;
  return own.finish();
}

extern "C" int rnt_buf_wrap(const rnt_ctx* ctx, void* device_ptr, size_t n_polys, int in_ntt,
                            rnt_buf** out) {
  if (!ctx || !device_ptr || !out) return fail(RNT_ERR_BAD_ARGUMENT, "null argument");
  if (n_polys == 0) return fail(RNT_ERR_BAD_ARGUMENT, "rnt_buf_wrap: empty batch");
  rnt_buf* b = new (std::nothrow) rnt_buf;
  if (!b) return fail(RNT_ERR_OUT_OF_MEMORY, "rnt_buf_wrap");
  b->ctx = ctx;
  b->n_polys = n_polys;
  b->data = device_ptr;
  b->in_ntt = in_ntt ? 1 : 0;
  b->owns = false;
  ctx_retain(ctx);
  *out = b;
  return RNT_OK;
}

extern "C" int rnt_buf_device_ptr(const rnt_buf* b, void** device_ptr, size_t* word_bytes_out) {
  if (!b || !device_ptr) return fail(RNT_ERR_BAD_ARGUMENT, "null argument");
  *device_ptr = b->data;
  if (word_bytes_out) *word_bytes_out = word_bytes(b->ctx->t.get());
  return RNT_OK;
}

extern "C" int rnt_buf_n_polys(const rnt_buf* b, size_t* n) {
  if (!b || !n) return fail(RNT_ERR_BAD_ARGUMENT, "null argument");
  *n = b->n_polys;
  return RNT_OK;
}
extern "C" int rnt_buf_is_ntt(const rnt_buf* b, int* in_ntt) {
  if (!b || !in_ntt) return fail(RNT_ERR_BAD_ARGUMENT, "null argument");
  *in_ntt = b->in_ntt;
  return RNT_OK;
}

extern "C" int rnt_upload(rnt_buf* b, const uint64_t* host, size_t n_polys, size_t channels,
                          int in_ntt) {
  if (int rc = check_buf(b, "rnt_upload")) return rc;
  if (!host) return fail(RNT_ERR_BAD_ARGUMENT, "rnt_upload: null host pointer");
  // from_channels order (poly.rs:78-93): channel count, then reducedness.
  if (channels != b->ctx->L)
    return fail_fields(RNT_ERR_CHANNEL_COUNT, b->ctx->L, channels,
                       "channel count mismatch: expected %zu, got %zu", b->ctx->L, channels);
  if (n_polys != b->n_polys)
    return fail(RNT_ERR_BAD_ARGUMENT, "rnt_upload: buffer holds %zu polys, got %zu", b->n_polys,
                n_polys);
  if (int rc = set_device(b->ctx)) return rc;
  rnt::Launch k = launch_for(b);
  const size_t words = poly_words(b);
  if (int rc = ensure_stage(b, words * 8 + 64)) return rc;
  unsigned long long* err = (unsigned long long*)((char*)b->stage + words * 8);
  HIP_TRY(hipMemcpyAsync(b->stage, host, words * 8, hipMemcpyHostToDevice, k.s), "hipMemcpy H2D");
  HIP_TRY(hipMemsetAsync(err, 0xff, 8, k.s), "hipMemset");
  LAUNCH(k.t, rnt::K_IMPORT, rnt::launch_import(k, b->data, (const uint64_t*)b->stage, in_ntt ? 1 : 0, err), "import");
  unsigned long long bad = 0;
  HIP_TRY(hipMemcpyAsync(&bad, err, 8, hipMemcpyDeviceToHost, k.s), "hipMemcpy D2H");
  HIP_TRY(hipStreamSynchronize(k.s), "hipStreamSynchronize");
  if (bad != ~0ull) {
    const size_t n = b->ctx->t->n;
    const size_t ch = (size_t)((bad / n) % b->ctx->L);
    // device data is now partially written; the reference returns Err and
    // builds no polynomial, so zero the buffer to keep it well-defined.
    cleanup(hipMemsetAsync(b->data, 0, words * word_bytes(k.t), k.s), "hipMemsetAsync(rejected upload)");
    cleanup(hipStreamSynchronize(k.s), "hipStreamSynchronize(rejected upload)");
    b->in_ntt = 0;
    return fail_fields(RNT_ERR_NON_REDUCED, host[bad], b->ctx->t->moduli[ch],
                       "coefficient %" PRIu64 " is not reduced modulo %" PRIu64, host[bad],
                       b->ctx->t->moduli[ch]);
  }
  b->in_ntt = in_ntt ? 1 : 0;
  trim_stage(b);
  return RNT_OK;
}

extern "C" int rnt_upload_coeffs(rnt_buf* b, const int64_t* coeffs, size_t n_polys) {
  if (int rc = check_buf(b, "rnt_upload_coeffs")) return rc;
  if (!coeffs) return fail(RNT_ERR_BAD_ARGUMENT, "rnt_upload_coeffs: null pointer");
  if (n_polys != b->n_polys)
    return fail(RNT_ERR_BAD_ARGUMENT, "rnt_upload_coeffs: buffer holds %zu polys, got %zu",
                b->n_polys, n_polys);
  if (int rc = set_device(b->ctx)) return rc;
  rnt::Launch k = launch_for(b);
  const size_t words = n_polys * b->ctx->t->n;
  if (int rc = ensure_stage(b, words * 8)) return rc;
  HIP_TRY(hipMemcpyAsync(b->stage, coeffs, words * 8, hipMemcpyHostToDevice, k.s), "hipMemcpy H2D");
  LAUNCH(k.t, rnt::K_IMPORT, rnt::launch_import_coeffs(k, b->data, (const int64_t*)b->stage), "import_coeffs");
  HIP_TRY(hipStreamSynchronize(k.s), "hipStreamSynchronize");
  b->in_ntt = 0;
  trim_stage(b);
  return RNT_OK;
}

extern "C" int rnt_download(const rnt_buf* cb, uint64_t* host, size_t n_polys) {
  rnt_buf* b = const_cast<rnt_buf*>(cb);  // staging only; contents unchanged
  if (int rc = check_buf(b, "rnt_download")) return rc;
  if (!host) return fail(RNT_ERR_BAD_ARGUMENT, "rnt_download: null host pointer");
  if (n_polys != b->n_polys)
    return fail(RNT_ERR_BAD_ARGUMENT, "rnt_download: buffer holds %zu polys, got %zu", b->n_polys,
                n_polys);
  if (int rc = set_device(b->ctx)) return rc;
  rnt::Launch k = launch_for(b);
  const size_t words = poly_words(b);
  if (int rc = ensure_stage(b, words * 8)) return rc;
  LAUNCH(k.t, rnt::K_EXPORT, rnt::launch_export(k, (uint64_t*)b->stage, b->data, b->in_ntt), "export");
  HIP_TRY(hipMemcpyAsync(host, b->stage, words * 8, hipMemcpyDeviceToHost, k.s), "hipMemcpy D2H");
  HIP_TRY(hipStreamSynchronize(k.s), "hipStreamSynchronize");
  trim_stage(b);
  return RNT_OK;
}

extern "C" int rnt_download_polys(const rnt_buf* cb, uint64_t* host, size_t first, size_t count) {
  rnt_buf* b = const_cast<rnt_buf*>(cb);  // staging only; contents unchanged
  if (int rc = check_buf(b, "rnt_download_polys")) return rc;
  if (!host) return fail(RNT_ERR_BAD_ARGUMENT, "rnt_download_polys: null host pointer");
  if (first > b->n_polys || count > b->n_polys - first)
    return fail(RNT_ERR_BAD_ARGUMENT, "rnt_download_polys: polys [%zu, %zu) outside a batch of %zu",
                first, first + count, b->n_polys);
  if (count == 0) return RNT_OK;
  if (int rc = set_device(b->ctx)) return rc;
  rnt::Launch k = launch_for(b);
  k.B = count;
  const size_t n = k.t->n, words = count * b->ctx->L * n;
  if (int rc = ensure_stage(b, words * 8)) return rc;
  const char* src = (const char*)b->data + first * n * word_bytes(k.t);
  LAUNCH(k.t, rnt::K_EXPORT, rnt::launch_export(k, (uint64_t*)b->stage, src, b->in_ntt, limb_stride(b)),
         "export");
  HIP_TRY(hipMemcpyAsync(host, b->stage, words * 8, hipMemcpyDeviceToHost, k.s), "hipMemcpy D2H");
  HIP_TRY(hipStreamSynchronize(k.s), "hipStreamSynchronize");
  trim_stage(b);
  return RNT_OK;
}

extern "C" int rnt_copy(rnt_buf* dst, const rnt_buf* src) {
  if (int rc = check_buf(dst, "rnt_copy")) return rc;
  if (int rc = check_buf(src, "rnt_copy")) return rc;
  if (int rc = check_same(dst, src, "rnt_copy")) return rc;
  if (dst == src) return RNT_OK;
  if (int rc = set_device(dst->ctx)) return rc;
  rnt::Launch k = launch_for(dst);
  const uint64_t bytes = poly_words(src) * word_bytes(k.t);
  if (bytes % 16 == 0 && ((uintptr_t)dst->data | (uintptr_t)src->data) % 16 == 0) {
    // a 16-byte-per-lane copy kernel: 6.0+ TB/s against hipMemcpyAsync's
    // 4.6 (bench.py's stream_copy_GBs times this)
    LAUNCH(k.t, rnt::K_COPY, rnt::launch_copy(k.s, dst->data, src->data, bytes), "copy");
  } else {
    HIP_TRY(hipMemcpyAsync(dst->data, src->data, bytes, hipMemcpyDeviceToDevice, k.s),
            "hipMemcpyAsync");
  }
  dst->in_ntt = src->in_ntt;
  return RNT_OK;
}

// ---------------------------------------------------------------------------
// ring ops
// ---------------------------------------------------------------------------
extern "C" int rnt_ntt_fwd(rnt_buf* b) {
  if (int rc = check_buf(b, "rnt_ntt_fwd")) return rc;
  if (b->in_ntt) return RNT_OK;  // poly.rs:137-139
  if (int rc = set_device(b->ctx)) return rc;
  rnt::Launch k = launch_for(b);
  const uint64_t ls = limb_stride(b);
  if (use_mf(k)) {
    // N = 2^16, u32 bases: the whole-plane MFMA transform (rnt_mfma.hip)
    LAUNCH(k.t, rnt::K_MF_NTT_FWD, rnt::launch_mf_ntt(k, 0, b->data, ls), "MFMA forward transform");
  } else if (rnt::whole_ok(k.t, 0)) {
    // 2^10 <= N <= 2^14: the whole transform in one row launch
    LAUNCH(k.t, rnt::K_WHOLE_FWD, rnt::launch_whole(k, 0, b->data, b->data, nullptr, ls), "whole-plane forward");
  } else {
    LAUNCH(k.t, rnt::K_COL_FWD, rnt::launch_col_fwd(k, b->data, b->data, nullptr, nullptr, ls, ls),
           "column forward");
    LAUNCH(k.t, rnt::K_ROW_FWD, rnt::launch_row(k, 0, b->data, nullptr, ls), "row forward");
  }
  b->in_ntt = 1;
  return RNT_OK;
}

extern "C" int rnt_ntt_inv(rnt_buf* b) {
  if (int rc = check_buf(b, "rnt_ntt_inv")) return rc;
  if (!b->in_ntt) return RNT_OK;  // poly.rs:155-157
  if (int rc = set_device(b->ctx)) return rc;
  if (int rc = to_coeff_into(b, b->data)) return rc;
  b->in_ntt = 0;
  return RNT_OK;
}

static long env_long(const char* name, long dflt) {
  const char* e = getenv(name);
  return e ? atol(e) : dflt;
}

extern "C" int rnt_mul(rnt_buf* out, const rnt_buf* a, const rnt_buf* b) {
  if (int rc = check_buf(out, "rnt_mul")) return rc;
  if (int rc = check_buf(a, "rnt_mul")) return rc;
  if (int rc = check_buf(b, "rnt_mul")) return rc;
  if (int rc = check_same(a, b, "rnt_mul")) return rc;
  if (int rc = check_same(out, a, "rnt_mul")) return rc;
  if (a->in_ntt != b->in_ntt)
    return fail(RNT_ERR_DOMAIN_MISMATCH, "mul_assign: domain mismatch (both must be in the same domain)");
  if (int rc = set_device(out->ctx)) return rc;
  rnt::Launch k = launch_for(out);
  if (a->in_ntt) {  // poly.rs:297-306
    LAUNCH(k.t, rnt::K_ELEMENTWISE, rnt::launch_elementwise(k, 3, out->data, a->data, b->data), "pointwise mul");
    out->in_ntt = 1;
    return RNT_OK;
  }
  // poly.rs:307-329: fwd(a), fwd(b), pointwise, inv -- three fused launches
  // over the whole batch: column passes of both operands (b's into the
  // workspace), the row kernel (both forward row passes, Montgomery
  // pointwise product, inverse rows), the inverse column pass.
  const uint64_t ls = limb_stride(out);
  if (rnt::whole_ok(k.t, 2)) {
    // 2^10 <= N <= 2^14: both transforms, the product and the inverse in
    // one row launch, 3 planes per (poly, limb)
    LAUNCH(k.t, rnt::K_WHOLE_MUL, rnt::launch_whole(k, 2, out->data, a->data, b->data, ls), "whole-plane product");
    out->in_ntt = 0;
    return RNT_OK;
  }
  if (rnt::plane_ok(k.t)) {
    const uint64_t planes = rnt::plane_scratch_planes((uint64_t)k.B * k.L);
    if (int rc = ensure_ws(out, planes * k.t->n * 4)) return rc;
    if (k.t->mf_mul && use_mf(k))
      LAUNCH(k.t, rnt::K_MF_MUL, rnt::launch_mf_mul(k, out->data, a->data, b->data, ls, out->ws),
             "matrix-core product");
    else
      LAUNCH(k.t, rnt::K_PLANE_FUSED, rnt::launch_plane_fused(k, out->data, a->data, b->data, out->ws, ls),
             "plane fused product");
    out->in_ntt = 0;
    return RNT_OK;
  }
  if (int rc = ensure_ws(out, poly_words(out) * word_bytes(k.t))) return rc;
  // lazy: the Harvey variant when every q < 2^30 (u32, Tables::lazy30) or
  // every q < 2^62 (u64, Tables::lazy62)
  LAUNCH(k.t, rnt::K_COL_FWD, rnt::launch_col_fwd(k, out->data, a->data, out->ws, b->data, ls, ls, true),
         "column forward");
  LAUNCH(k.t, rnt::K_ROW_MUL, rnt::launch_row(k, 2, out->data, out->ws, ls, true), "row mul");
  LAUNCH(k.t, rnt::K_COL_INV,
         rnt::launch_col_inv(k, out->data, ls, out->data, ls, rnt::mul_truncated(k.t) ? 2 : 1, nullptr, true),
         "column inverse");
  out->in_ntt = 0;
  return RNT_OK;
}

static int binary_elementwise(rnt_buf* out, const rnt_buf* a, const rnt_buf* b, int op,
                              const char* name) {
  if (int rc = check_buf(out, name)) return rc;
  if (int rc = check_buf(a, name)) return rc;
  if (int rc = check_buf(b, name)) return rc;
  if (int rc = check_same(a, b, name)) return rc;
  if (int rc = check_same(out, a, name)) return rc;
  if (a->in_ntt != b->in_ntt) return fail(RNT_ERR_DOMAIN_MISMATCH, "%s: domain mismatch", name);
  if (int rc = set_device(out->ctx)) return rc;
  rnt::Launch k = launch_for(out);
  LAUNCH(k.t, rnt::K_ELEMENTWISE, rnt::launch_elementwise(k, op, out->data, a->data, b->data), name);
  out->in_ntt = a->in_ntt;
  return RNT_OK;
}

extern "C" int rnt_add(rnt_buf* out, const rnt_buf* a, const rnt_buf* b) {
  return binary_elementwise(out, a, b, 0, "add_assign");
}
extern "C" int rnt_sub(rnt_buf* out, const rnt_buf* a, const rnt_buf* b) {
  return binary_elementwise(out, a, b, 1, "sub");
}
extern "C" int rnt_neg(rnt_buf* out, const rnt_buf* a) {
  if (int rc = check_buf(out, "rnt_neg")) return rc;
  if (int rc = check_buf(a, "rnt_neg")) return rc;
  if (int rc = check_same(out, a, "rnt_neg")) return rc;
  if (int rc = set_device(out->ctx)) return rc;
  rnt::Launch k = launch_for(out);
  LAUNCH(k.t, rnt::K_ELEMENTWISE, rnt::launch_elementwise(k, 2, out->data, a->data, nullptr), "neg");
  out->in_ntt = a->in_ntt;
  return RNT_OK;
}

extern "C" int rnt_rescale(rnt_buf* out, const rnt_buf* in) {
  if (int rc = check_buf(out, "rnt_rescale")) return rc;
  if (int rc = check_buf(in, "rnt_rescale")) return rc;
  const size_t L = in->ctx->L;
  if (L < 2)  // poly.rs:191-197
    return fail_fields(RNT_ERR_INVALID_MOD_DROP, 1, L, "invalid mod-drop count 1 for %zu channels", L);
  if (out->ctx->t != in->ctx->t || out->ctx->L != L - 1)
    return fail(RNT_ERR_BASIS_MISMATCH, "rescale: output basis is not drop_last(1) of the input's");
  if (out->n_polys != in->n_polys)
    return fail(RNT_ERR_BAD_ARGUMENT, "rescale: batch sizes differ");
  if (int rc = set_device(in->ctx)) return rc;
  rnt::Launch k = launch_for(in);
  const void* src = in->data;
  if (in->in_ntt) {  // poly.rs:199-210: clone + to_coeff_domain
    if (int rc = ensure_ws(out, poly_words(in) * word_bytes(k.t))) return rc;
    if (int rc = to_coeff_into(in, out->ws)) return rc;
    src = out->ws;
  }
  LAUNCH(k.t, rnt::K_RESCALE, rnt::launch_rescale(k, out->data, src), "rescale");
  out->in_ntt = 0;
  return RNT_OK;
}

// Device constants {inv[L], invp[L]} for rescaling by an external modulus.
static int resc_ext_table(const rnt_ctx* ctx, uint64_t q_last, const void** inv, const void** invp) {
  rnt::Tables* t = ctx->t.get();
  const size_t Lr = t->L;  // table covers every limb of the root basis
  std::lock_guard<std::mutex> g(t->resc_mu);
  for (auto& e : t->resc_ext)
    if (e.first == q_last) {
      *inv = e.second;
      *invp = (const char*)e.second + Lr * word_bytes(t);
      return RNT_OK;
    }
  const unsigned wbits = t->wide ? 64 : 32;
  std::vector<uint64_t> h(2 * Lr);
  for (size_t l = 0; l < Lr; ++l) {
    const uint64_t ql = t->moduli[l];
    if (ql == q_last) {  // the limb being dropped: never read
      h[l] = h[Lr + l] = 0;
      continue;
    }
    const uint64_t v = rnt::host::invmod(q_last % ql, ql);
    if (v == 0)
      return fail(RNT_ERR_BAD_ARGUMENT, "rescale: modulus %" PRIu64 " is not coprime to %" PRIu64, q_last, ql);
    h[l] = v;
    h[Lr + l] = rnt::host::shoup_companion(v, ql, wbits);
  }
  void* d = nullptr;
  const size_t wb = word_bytes(t);
  HIP_TRY(hipMalloc(&d, 2 * Lr * wb), "hipMalloc(rescale constants)");
  if (wb == 4) {
    std::vector<uint32_t> h32(h.begin(), h.end());
    HIP_TRY(hipMemcpy(d, h32.data(), 2 * Lr * 4, hipMemcpyHostToDevice), "hipMemcpy");
  } else {
    HIP_TRY(hipMemcpy(d, h.data(), 2 * Lr * 8, hipMemcpyHostToDevice), "hipMemcpy");
  }
  t->resc_ext.push_back({q_last, d});
  *inv = d;
  *invp = (const char*)d + Lr * wb;
  return RNT_OK;
}

extern "C" int rnt_rescale_ext(rnt_buf* out, const rnt_buf* in, const void* last_limb,
                               uint64_t q_last) {
  if (int rc = check_buf(out, "rnt_rescale_ext")) return rc;
  if (int rc = check_buf(in, "rnt_rescale_ext")) return rc;
  if (!last_limb) return fail(RNT_ERR_BAD_ARGUMENT, "rnt_rescale_ext: null last limb");
  if (in->in_ntt)
    return fail(RNT_ERR_DOMAIN_MISMATCH, "rnt_rescale_ext: input must be in coefficient domain");
  const size_t L = in->ctx->L;
  const rnt::Tables* t = in->ctx->t.get();
  // the owner of q_last drops it; every other shard keeps all its limbs
  const size_t keep = (L > 0 && t->moduli[L - 1] == q_last) ? L - 1 : L;
  if (keep == 0)
    return fail_fields(RNT_ERR_INVALID_MOD_DROP, 1, L, "rescale: nothing left after dropping the last limb");
  if (out->ctx->t != in->ctx->t || out->ctx->L != keep)
    return fail(RNT_ERR_BASIS_MISMATCH, "rnt_rescale_ext: output basis must keep %zu limbs of the input's", keep);
  if (out->n_polys != in->n_polys)
    return fail(RNT_ERR_BAD_ARGUMENT, "rnt_rescale_ext: batch sizes differ");
  if (int rc = set_device(in->ctx)) return rc;
  const void* inv = nullptr;
  const void* invp = nullptr;
  if (int rc = resc_ext_table(in->ctx, q_last, &inv, &invp)) return rc;
  rnt::Launch k = launch_for(in);
  k.L = keep;
  LAUNCH(k.t, rnt::K_RESCALE, rnt::launch_rescale_ext(k, out->data, in->data, last_limb, inv, invp),
         "rescale_ext");
  out->in_ntt = 0;
  return RNT_OK;
}

// ---- decode-side CRT (basis.rs:158-180, poly.rs:404-427) ----------------

namespace {

// Little-endian 32-bit-word big integers for the host-side constants.
using Big = std::vector<uint32_t>;
void big_mul_small(Big& a, uint64_t m) {
  // a *= m (m < 2^64), growing a
  const uint32_t mlo = (uint32_t)m, mhi = (uint32_t)(m >> 32);
  Big r(a.size() + 2, 0);
  for (int half = 0; half < 2; ++half) {
    const uint64_t f = half ? mhi : mlo;
    if (!f) continue;
    uint64_t carry = 0;
    for (size_t w = 0; w < a.size(); ++w) {
      const uint64_t t = (uint64_t)a[w] * f + r[w + half] + carry;
      r[w + half] = (uint32_t)t;
      carry = t >> 32;
    }
    for (size_t w = a.size() + half; carry && w < r.size(); ++w) {
      const uint64_t t = (uint64_t)r[w] + carry;
      r[w] = (uint32_t)t;
      carry = t >> 32;
    }
  }
  while (r.size() > 1 && r.back() == 0) r.pop_back();
  a.swap(r);
}

}  // namespace

// Constants of the centred CRT for the first L limbs of a basis, cached per
// (tables, L): device block {qi_words[L][MW], q[MW], qh[MW], inv[L],
// inv_p[L], rq[L]} and the CrtConsts pointing into it.
static int crt_tables(const rnt_ctx* ctx, const void** consts, uint32_t* mw_out) {
  rnt::Tables* t = ctx->t.get();
  const size_t L = ctx->L;
  std::lock_guard<std::mutex> g(t->resc_mu);
  for (auto& e : t->crt_cache)
    if (e.first == L) {
      *consts = &e.second.cc;
      *mw_out = e.second.mw;
      return RNT_OK;
    }
  Big Q{1};
  for (size_t l = 0; l < L; ++l) big_mul_small(Q, t->moduli[l]);
  uint32_t mw = 4;
  while (mw < Q.size()) mw *= 2;
  if (mw > 128) return fail(RNT_ERR_BAD_ARGUMENT, "CRT: Q has %zu 32-bit words (max 128)", Q.size());
  std::vector<uint32_t> qi(L * mw, 0), qw(mw, 0), qh(mw, 0);
  std::vector<uint64_t> inv(L), invp(L);
  std::vector<double> rq(L);
  const unsigned wbits = t->wide ? 64 : 32;
  for (size_t l = 0; l < L; ++l) {
    Big Ql{1};
    uint64_t ql_mod = 1;  // (Q/q_l) mod q_l
    for (size_t m = 0; m < L; ++m) {
      if (m == l) continue;
      big_mul_small(Ql, t->moduli[m]);
      ql_mod = rnt::host::mulmod(ql_mod, t->moduli[m] % t->moduli[l], t->moduli[l]);
    }
    for (size_t w = 0; w < Ql.size() && w < mw; ++w) qi[l * mw + w] = Ql[w];
    inv[l] = rnt::host::invmod(ql_mod, t->moduli[l]);
    if (inv[l] == 0 && L > 1)
      return fail(RNT_ERR_BAD_ARGUMENT, "CRT: moduli are not pairwise coprime");
    if (L == 1) inv[l] = 1;
    invp[l] = rnt::host::shoup_companion(inv[l], t->moduli[l], wbits);
    rq[l] = 1.0 / (double)t->moduli[l];
  }
  for (size_t w = 0; w < Q.size(); ++w) qw[w] = Q[w];
  for (size_t w = 0; w < mw; ++w) qh[w] = (qw[w] >> 1) | (w + 1 < mw ? qw[w + 1] << 31 : 0);
  const size_t bytes = (L * mw + 2 * mw) * 4 + L * 8 * 2 + L * 8;
  void* d = nullptr;
  HIP_TRY(hipMalloc(&d, bytes), "hipMalloc(CRT constants)");
  std::vector<unsigned char> h(bytes);
  size_t off = 0;
  auto put = [&](const void* src, size_t n) {
    memcpy(h.data() + off, src, n);
    off += n;
  };
  rnt::CrtDev cd;
  cd.dev = d;
  cd.mw = mw;
  cd.cc.qi_words = (const uint32_t*)((char*)d + off);
  put(qi.data(), qi.size() * 4);
  cd.cc.q_words = (const uint32_t*)((char*)d + off);
  put(qw.data(), mw * 4);
  cd.cc.qh_words = (const uint32_t*)((char*)d + off);
  put(qh.data(), mw * 4);
  cd.cc.inv = (const uint64_t*)((char*)d + off);
  put(inv.data(), L * 8);
  cd.cc.inv_p = (const uint64_t*)((char*)d + off);
  put(invp.data(), L * 8);
  cd.cc.rq = (const double*)((char*)d + off);
  put(rq.data(), L * 8);
  HIP_TRY(hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice), "hipMemcpy(CRT constants)");
  t->crt_cache.push_back({L, cd});
  *consts = &t->crt_cache.back().second.cc;
  *mw_out = mw;
  return RNT_OK;
}

static int crt_download(const rnt_buf* cb, uint64_t* host, size_t n_polys, size_t out_words,
                        const char* name) {
  rnt_buf* b = const_cast<rnt_buf*>(cb);  // workspace / staging only
  if (int rc = check_buf(b, name)) return rc;
  if (!host) return fail(RNT_ERR_BAD_ARGUMENT, "%s: null host pointer", name);
  if (n_polys != b->n_polys)
    return fail(RNT_ERR_BAD_ARGUMENT, "%s: buffer holds %zu polys, got %zu", name, b->n_polys, n_polys);
  if (out_words == 0 || out_words > 64) return fail(RNT_ERR_BAD_ARGUMENT, "%s: 1..64 words", name);
  if (int rc = set_device(b->ctx)) return rc;
  const void* consts = nullptr;
  uint32_t mw = 0;
  if (int rc = crt_tables(b->ctx, &consts, &mw)) return rc;
  rnt::Launch k = launch_for(b);
  const void* src = b->data;
  if (b->in_ntt) {  // poly.rs:408-417: a coefficient-domain clone
    if (int rc = ensure_ws(b, poly_words(b) * word_bytes(k.t))) return rc;
    if (int rc = to_coeff_into(b, b->ws)) return rc;
    src = b->ws;
  }
  const size_t coeffs = b->n_polys * k.t->n;
  if (int rc = ensure_stage(b, coeffs * out_words * 8)) return rc;
  LAUNCH(k.t, rnt::K_CRT, rnt::launch_crt(k, (uint64_t*)b->stage, src, consts, mw, (uint32_t)out_words),
         "crt");
  HIP_TRY(hipMemcpyAsync(host, b->stage, coeffs * out_words * 8, hipMemcpyDeviceToHost, k.s),
          "hipMemcpy D2H");
  HIP_TRY(hipStreamSynchronize(k.s), "hipStreamSynchronize");
  trim_stage(b);
  return RNT_OK;
}

extern "C" int rnt_to_coeffs(const rnt_buf* buf, int64_t* host, size_t n_polys) {
  return crt_download(buf, (uint64_t*)host, n_polys, 1, "rnt_to_coeffs");
}

extern "C" int rnt_crt_centered(const rnt_buf* buf, uint64_t* host, size_t n_polys, size_t words) {
  return crt_download(buf, host, n_polys, words, "rnt_crt_centered");
}

// ---------------------------------------------------------------------------
// samplers (PolySampler, traits.rs:74-127; rnt_sample.hip)
// ---------------------------------------------------------------------------
static int sample_into(rnt_buf* out, int kind, double sigma, size_t h, uint64_t seed,
                       uint64_t stream, const char* name) {
  if (int rc = set_device(out->ctx)) return rc;
  rnt::Launch k = launch_for(out);
  rnt::SampleKey s;
  s.k0 = (uint32_t)seed;
  s.k1 = (uint32_t)(seed >> 32) ^ (uint32_t)(stream >> 32);
  s.stream = (uint32_t)stream;
  LAUNCH(k.t, rnt::K_SAMPLE, rnt::launch_sample(k, kind, out->data, s, sigma, (uint32_t)h), name);
  out->in_ntt = 0;
  return RNT_OK;
}

extern "C" int rnt_sample_uniform(rnt_buf* out, uint64_t seed, uint64_t stream) {
  if (int rc = check_buf(out, "rnt_sample_uniform")) return rc;
  return sample_into(out, 0, 0.0, 0, seed, stream, "sample_uniform");
}

extern "C" int rnt_sample_gaussian(rnt_buf* out, double std_dev, uint64_t seed, uint64_t stream) {
  if (int rc = check_buf(out, "rnt_sample_gaussian")) return rc;
  // poly.rs:452-453 / sampling.rs:31-45 panic on these
  if (!(std_dev > 0.0) || !std::isfinite(std_dev))
    return fail(RNT_ERR_BAD_ARGUMENT, "sample_gaussian: std_dev must be finite and positive");
  return sample_into(out, 1, std_dev, 0, seed, stream, "sample_gaussian");
}

extern "C" int rnt_sample_ternary(rnt_buf* out, size_t hamming_weight, uint64_t seed,
                                  uint64_t stream) {
  if (int rc = check_buf(out, "rnt_sample_ternary")) return rc;
  // sampling.rs:71-80 panics on an oversized Hamming weight
  if (hamming_weight > out->ctx->t->n)
    return fail(RNT_ERR_BAD_ARGUMENT, "sample_tribits: hamming weight %zu exceeds degree %zu",
                hamming_weight, out->ctx->t->n);
  return sample_into(out, 2, 0.0, hamming_weight, seed, stream, "sample_tribits");
}

// ---------------------------------------------------------------------------
// CKKS encoder / decoder (ckks_encoder.rs:85-156, special_fft.rs; the
// special FFT in rnt_encode.hip)
// ---------------------------------------------------------------------------
static int sfft_table(const rnt_ctx* ctx, const void** tab) {
  rnt::Tables* t = ctx->t.get();
  std::lock_guard<std::mutex> g(t->sfft_mu);
  if (!t->sfft_tw) {
    const std::vector<double> h = rnt::sfft_twiddles(t->log_n);
    void* d = nullptr;
    HIP_TRY(hipMalloc(&d, h.size() * sizeof(double)), "hipMalloc(sfft twiddles)");
    const hipError_t e = hipMemcpy(d, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      cleanup(hipFree(d), "hipFree(sfft twiddles)");
      return hip_fail(e, "hipMemcpy(sfft twiddles)");
    }
    t->sfft_tw = d;
  }
  *tab = t->sfft_tw;
  return RNT_OK;
}

static int sfft_check(const rnt_buf* b, const double* values, size_t n_values,
                      uint32_t scale_bits, const char* name) {
  if (int rc = check_buf(b, name)) return rc;
  const size_t n = b->ctx->t->n;
  if (!rnt::sfft_supported(b->ctx->t->log_n))
    return fail(RNT_ERR_BAD_ARGUMENT, "%s: degree %zu has no slots", name, n);
  // ckks_encoder.rs:70-75 (a panic in the reference)
  if (n_values > n / 2)
    return fail(RNT_ERR_BAD_ARGUMENT, "%s: %zu values exceed max slots %zu", name, n_values, n / 2);
  if (n_values && b->n_polys && !values) return fail(RNT_ERR_BAD_ARGUMENT, "%s: null values", name);
  // ckks_encoder.rs:43 asserts scale_bits > 0; 2^scale_bits must be a finite f64
  if (scale_bits == 0 || scale_bits > 1000)
    return fail(RNT_ERR_BAD_ARGUMENT, "%s: scale_bits must be in [1, 1000], got %u", name, scale_bits);
  return RNT_OK;
}

extern "C" int rnt_encode(rnt_buf* out, const double* values, size_t n_values, uint32_t scale_bits) {
  if (int rc = sfft_check(out, values, n_values, scale_bits, "rnt_encode")) return rc;
  if (int rc = set_device(out->ctx)) return rc;
  const void* tw = nullptr;
  if (int rc = sfft_table(out->ctx, &tw)) return rc;
  rnt::Launch k = launch_for(out);
  const size_t B = out->n_polys, n = k.t->n;
  if (B == 0) {
    out->in_ntt = 0;
    return RNT_OK;
  }
  // stage: the slot values in, then the rounded i64 coefficients;
  // ws: [B][N/2] complex working planes
  if (int rc = ensure_stage(out, B * n * 8)) return rc;
  if (int rc = ensure_ws(out, B * n * 8)) return rc;
  if (n_values)
    HIP_TRY(hipMemcpyAsync(out->stage, values, B * n_values * 16, hipMemcpyHostToDevice, k.s),
            "hipMemcpy H2D");
  LAUNCH(k.t, rnt::K_SFFT,
         rnt::launch_sfft_encode(k, (int64_t*)out->stage, out->ws, out->stage, (uint32_t)n_values,
                                 scale_bits, tw),
         "special fft (encode)");
  LAUNCH(k.t, rnt::K_IMPORT, rnt::launch_import_coeffs(k, out->data, (const int64_t*)out->stage),
         "import_coeffs");
  HIP_TRY(hipStreamSynchronize(k.s), "hipStreamSynchronize");
  out->in_ntt = 0;
  trim_stage(out);
  return RNT_OK;
}

extern "C" int rnt_decode(const rnt_buf* cb, double* values, size_t n_values, uint32_t scale_bits) {
  rnt_buf* b = const_cast<rnt_buf*>(cb);  // workspace / staging only
  if (int rc = sfft_check(b, values, n_values, scale_bits, "rnt_decode")) return rc;
  if (int rc = set_device(b->ctx)) return rc;
  const void* tw = nullptr;
  if (int rc = sfft_table(b->ctx, &tw)) return rc;
  const void* consts = nullptr;
  uint32_t mw = 0;
  if (int rc = crt_tables(b->ctx, &consts, &mw)) return rc;
  rnt::Launch k = launch_for(b);
  const size_t B = b->n_polys, n = k.t->n;
  if (B == 0 || n_values == 0) return RNT_OK;
  // ws holds the coefficient-domain clone of an NTT-domain input, then the
  // complex planes; stage the centred i64 coefficients (to_coeffs)
  if (int rc = ensure_ws(b, std::max(poly_words(b) * word_bytes(k.t), B * n * 8))) return rc;
  if (int rc = ensure_stage(b, B * n * 8)) return rc;
  const void* src = b->data;
  if (b->in_ntt) {  // poly.rs:408-417: a coefficient-domain clone
    if (int rc = to_coeff_into(b, b->ws)) return rc;
    src = b->ws;
  }
  LAUNCH(k.t, rnt::K_CRT, rnt::launch_crt(k, (uint64_t*)b->stage, src, consts, mw, 1), "crt");
  LAUNCH(k.t, rnt::K_SFFT,
         rnt::launch_sfft_decode(k, b->ws, (const int64_t*)b->stage, scale_bits, tw),
         "special fft (decode)");
  HIP_TRY(hipMemcpy2DAsync(values, n_values * 16, b->ws, (n / 2) * 16, n_values * 16, B,
                           hipMemcpyDeviceToHost, k.s),
          "hipMemcpy2D D2H");
  HIP_TRY(hipStreamSynchronize(k.s), "hipStreamSynchronize");
  trim_stage(b);
  return RNT_OK;
}

extern "C" int rnt_mod_drop_last(rnt_buf* out, const rnt_buf* in) {
  if (int rc = check_buf(out, "rnt_mod_drop_last")) return rc;
  if (int rc = check_buf(in, "rnt_mod_drop_last")) return rc;
  if (out->ctx->t != in->ctx->t || out->ctx->L > in->ctx->L)
    return fail(RNT_ERR_BASIS_MISMATCH, "mod_drop_last: output basis is not a prefix of the input's");
  if (out->n_polys != in->n_polys)
    return fail(RNT_ERR_BAD_ARGUMENT, "mod_drop_last: batch sizes differ");
  if (int rc = set_device(in->ctx)) return rc;
  rnt::Launch k = launch_for(out);
  // [L][B][N]: the kept channels are a contiguous prefix
  if (out != in)
    HIP_TRY(hipMemcpyAsync(out->data, in->data, poly_words(out) * word_bytes(k.t),
                           hipMemcpyDeviceToDevice, k.s),
            "hipMemcpyAsync");
  out->in_ntt = in->in_ntt;
  return RNT_OK;
}

extern "C" int rnt_automorphism(rnt_buf* out, const rnt_buf* in, uint64_t g) {
  if (int rc = check_buf(out, "rnt_automorphism")) return rc;
  if (int rc = check_buf(in, "rnt_automorphism")) return rc;
  if (int rc = check_same(out, in, "rnt_automorphism")) return rc;
  if (int rc = set_device(in->ctx)) return rc;
  rnt::Launch k = launch_for(in);
  const uint64_t two_n = 2 * (uint64_t)k.t->n;
  if (g % two_n == 0) return rnt_copy(out, in);  // poly.rs:508-511: self.clone()
  const void* src = in->data;
  if (in->in_ntt || out == in) {
    if (int rc = ensure_ws(out, poly_words(in) * word_bytes(k.t))) return rc;
    if (in->in_ntt) {
      if (int rc = to_coeff_into(in, out->ws)) return rc;
    } else {
      HIP_TRY(hipMemcpyAsync(out->ws, in->data, poly_words(in) * word_bytes(k.t),
                             hipMemcpyDeviceToDevice, k.s),
              "hipMemcpyAsync");
    }
    src = out->ws;
  }
  LAUNCH(k.t, rnt::K_AUTOMORPHISM, rnt::launch_automorphism(k, out->data, src, g), "automorphism");
  out->in_ntt = 0;
  return RNT_OK;
}

static uint64_t rotation_exponent(int32_t k, uint64_t two_n) {
  // poly.rs:546-569: 5^|k| mod 2N, and for k < 0 the composition with
  // X -> X^(2N-1): both are odd, so the two automorphisms compose exactly
  // into one with exponent 5^|k| * (2N-1) mod 2N.
  const uint64_t r = k >= 0 ? (uint64_t)k : (uint64_t)(-(int64_t)k);
  uint64_t e = rnt::host::powmod(5, r, two_n);
  if (k < 0) e = rnt::host::mulmod(e, two_n - 1, two_n);
  return e;
}

extern "C" int rnt_rotate_slots(rnt_buf* out, const rnt_buf* in, int32_t k) {
  if (int rc = check_buf(in, "rnt_rotate_slots")) return rc;
  return rnt_automorphism(out, in, rotation_exponent(k, 2 * (uint64_t)in->ctx->t->n));
}

// ---------------------------------------------------------------------------
// key-switching
// ---------------------------------------------------------------------------
extern "C" int rnt_key_prepare(rnt_buf* key_a, rnt_buf* key_b) {
  if (int rc = check_buf(key_a, "rnt_key_prepare")) return rc;
  if (int rc = check_buf(key_b, "rnt_key_prepare")) return rc;
  if (int rc = check_same(key_a, key_b, "rnt_key_prepare")) return rc;
  // one poly per SOURCE limb: the basis' own channel count for rnt_keyswitch,
  // the global count for a limb shard's rnt_keyswitch_ext (checked there)
  if (key_a->n_polys != key_b->n_polys)
    return fail_fields(RNT_ERR_CHANNEL_COUNT, key_a->n_polys, key_b->n_polys,
                       "gadget key halves differ: %zu vs %zu polys", key_a->n_polys, key_b->n_polys);
  if (int rc = rnt_ntt_fwd(key_a)) return rc;
  return rnt_ntt_fwd(key_b);
}

namespace {

int check_key(const rnt_buf* d, const rnt_buf* key_a, const rnt_buf* key_b) {
  if (int rc = check_buf(key_a, "key")) return rc;
  if (int rc = check_buf(key_b, "key")) return rc;
  if (key_a->ctx != d->ctx || key_b->ctx != d->ctx)
    return fail(RNT_ERR_BASIS_MISMATCH, "key-switch: key and ciphertext belong to different bases");
  if (key_a->n_polys != d->ctx->L || key_b->n_polys != d->ctx->L)
    return fail_fields(RNT_ERR_CHANNEL_COUNT, d->ctx->L,
                       key_a->n_polys != d->ctx->L ? key_a->n_polys : key_b->n_polys,
                       "gadget key must hold one poly per channel (%zu)", d->ctx->L);
  if (!key_a->in_ntt || !key_b->in_ntt)
    return fail(RNT_ERR_DOMAIN_MISMATCH, "key-switch: keys must be prepared (rnt_key_prepare)");
  return RNT_OK;
}

// polys per key-switch chunk so that S ([L][L][Bc][N]) stays <= ~1 GiB
// Key-switch workspace cap: S ([L][L][Bc][N] words) of a chunk.  The key
// rows are read once per chunk from HBM (the batch hits them in cache, see
// row_pos_pfast), so bigger chunks cut key traffic per ciphertext; 4 GiB is
// a small slice of the 288 GB.
size_t ks_chunk(const rnt::Tables* t, size_t L, size_t B) {
  // (the whole-plane key-switch has no S: its chunk is bounded by the
  // ct-mul's seven chunk-local planes per limb instead)
  const size_t per = (rnt::ks_whole_ok(t) ? 7 * L : L * L) * t->n * (t->wide ? 8 : 4);
  size_t c = t->ks_ws_bytes;
  c = per ? c / per : B;
  if (c < 1) c = 1;
  return std::min(c, B);
}

// Key-switch scratch of a chunk of bc polys (words): S | U0 | U1, or none
// for the whole-plane key-switch.
size_t ks_scratch_words(const rnt::Tables* t, size_t L, size_t bc) {
  return rnt::ks_whole_ok(t) ? 0 : (L * L + 2 * L) * bc * t->n;
}

// Decomposition + key-switch rows of one chunk (k.B polys, k.L target limbs,
// k.src_limbs() source limbs at src) into the NTT-row accumulators U0/U1.
// (Running them per group of target limbs, so each S slice could stay in the
// Infinity Cache between the two kernels, was slower: profiles/r02_ab_ks_groups.txt.)
int ks_decompose_rows(const rnt::Launch& k, char* S, const char* src, uint64_t src_ls, char* U0,
                      char* U1, uint64_t u_ls, const rnt_buf* key_a, const rnt_buf* key_b,
                      const char* i0, const char* i1, uint64_t init_ls) {
  LAUNCH(k.t, rnt::K_KS_DECOMPOSE, rnt::launch_ks_decompose(k, S, src, src_ls), "ks decompose");
  LAUNCH(k.t, rnt::K_KS_ROWS,
         rnt::launch_ks_rows(k, U0, U1, u_ls, S, key_a->data, key_b->data, limb_stride(key_a), i0, i1,
                             init_ls),
         "ks rows");
  return RNT_OK;
}

// Gadget sum for polys [p0, p0+bc) of d into out0/out1 (full-batch layout):
// out0 = INV(sum_i NTT(alpha_i) key_b[i] + init0) (+ add0), etc.
// ws layout: S | U0 | U1.
int ks_chunk_run(rnt::Launch k, void* ws, const rnt_buf* d, size_t p0, size_t bc,
                 const rnt_buf* key_a, const rnt_buf* key_b, void* out0, void* out1,
                 uint64_t out_ls, const void* init0, const void* init1, uint64_t init_ls,
                 const void* add0, int with_init) {
  const size_t n = k.t->n, L = k.L, wb = k.t->wide ? 8 : 4;
  k.B = bc;
  if (rnt::ks_whole_ok(k.t)) {
    // 2^10 <= N <= 2^14: one launch, no S (ws unused)
    const char* i0 = with_init && init0 ? (const char*)init0 + p0 * n * wb : nullptr;
    const char* i1 = with_init && init1 ? (const char*)init1 + p0 * n * wb : nullptr;
    const char* a0 = add0 ? (const char*)add0 + p0 * n * wb : nullptr;
    LAUNCH(k.t, rnt::K_KS_WHOLE,
           rnt::launch_ks_whole(k, (char*)out0 + p0 * n * wb, (char*)out1 + p0 * n * wb, out_ls,
                                (const char*)d->data + p0 * n * wb, limb_stride(d), key_a->data, key_b->data,
                                limb_stride(key_a), i0, i1, init_ls, a0),
           "whole-plane key-switch");
    return RNT_OK;
  }
  char* S = (char*)ws;
  char* U0 = S + L * L * bc * n * wb;
  char* U1 = U0 + L * bc * n * wb;
  const uint64_t cls = (uint64_t)bc * n;  // chunk-local limb stride
  const uint64_t d_ls = limb_stride(d);
  const char* i0 = with_init && init0 ? (const char*)init0 + p0 * n * wb : nullptr;
  const char* i1 = with_init && init1 ? (const char*)init1 + p0 * n * wb : nullptr;
  if (int rc = ks_decompose_rows(k, S, (const char*)d->data + p0 * n * wb, d_ls, U0, U1, cls, key_a,
                                 key_b, i0, i1, init_ls))
    return rc;
  const char* a0 = add0 ? (const char*)add0 + p0 * n * wb : nullptr;
  LAUNCH(k.t, rnt::K_COL_INV, rnt::launch_col_inv(k, (char*)out0 + p0 * n * wb, out_ls, U0, cls, 1, a0), "ks inverse");
  LAUNCH(k.t, rnt::K_COL_INV, rnt::launch_col_inv(k, (char*)out1 + p0 * n * wb, out_ls, U1, cls, 1, nullptr), "ks inverse");
  return RNT_OK;
}

}  // namespace

extern "C" int rnt_keyswitch(rnt_buf* acc0, rnt_buf* acc1, const rnt_buf* d, const rnt_buf* key_a,
                             const rnt_buf* key_b) {
  if (int rc = check_buf(acc0, "rnt_keyswitch")) return rc;
  if (int rc = check_buf(acc1, "rnt_keyswitch")) return rc;
  if (int rc = check_buf(d, "rnt_keyswitch")) return rc;
  if (int rc = check_same(acc0, d, "rnt_keyswitch")) return rc;
  if (int rc = check_same(acc1, d, "rnt_keyswitch")) return rc;
  if (int rc = check_key(d, key_a, key_b)) return rc;
  if (d->in_ntt) return fail(RNT_ERR_DOMAIN_MISMATCH, "key-switch input must be in coefficient domain");
  if (acc0 == acc1 || acc0 == d || acc1 == d)
    return fail(RNT_ERR_BAD_ARGUMENT, "rnt_keyswitch: outputs must not alias each other or d");
  if (int rc = set_device(d->ctx)) return rc;
  rnt::Launch k = launch_for(d);
  const size_t L = k.L, wb = word_bytes(k.t);
  const size_t bc = ks_chunk(k.t, L, d->n_polys);
  CallWs ws(acc0);
  if (int rc = ws.get(std::max<size_t>(ks_scratch_words(k.t, L, bc) * wb, 16))) return rc;
  for (size_t p0 = 0; p0 < d->n_polys; p0 += bc) {
    const size_t c = std::min(bc, d->n_polys - p0);
    if (int rc = ks_chunk_run(k, ws.p, d, p0, c, key_a, key_b, acc0->data, acc1->data,
                              limb_stride(d), nullptr, nullptr, 0, nullptr, 0))
      return rc;
  }
  acc0->in_ntt = acc1->in_ntt = 0;
  return RNT_OK;
}

extern "C" int rnt_keyswitch_ext(rnt_buf* acc0, rnt_buf* acc1, const void* src, size_t src_limbs,
                                 const rnt_buf* key_a, const rnt_buf* key_b, const rnt_buf* init0,
                                 const rnt_buf* init1) {
  if (int rc = check_buf(acc0, "rnt_keyswitch_ext")) return rc;
  if (int rc = check_buf(acc1, "rnt_keyswitch_ext")) return rc;
  if (int rc = check_same(acc0, acc1, "rnt_keyswitch_ext")) return rc;
  if (!src || src_limbs == 0) return fail(RNT_ERR_BAD_ARGUMENT, "rnt_keyswitch_ext: empty source");
  if (int rc = check_buf(key_a, "key")) return rc;
  if (int rc = check_buf(key_b, "key")) return rc;
  if (key_a->ctx != acc0->ctx || key_b->ctx != acc0->ctx)
    return fail(RNT_ERR_BASIS_MISMATCH, "key-switch: key and accumulator belong to different bases");
  if (key_a->n_polys != src_limbs || key_b->n_polys != src_limbs)
    return fail_fields(RNT_ERR_CHANNEL_COUNT, src_limbs,
                       key_a->n_polys != src_limbs ? key_a->n_polys : key_b->n_polys,
                       "gadget key must hold one poly per source limb (%zu)", src_limbs);
  if (!key_a->in_ntt || !key_b->in_ntt)
    return fail(RNT_ERR_DOMAIN_MISMATCH, "key-switch: keys must be prepared (rnt_key_prepare)");
  const rnt_buf* seeds[2] = {init0, init1};
  for (const rnt_buf* sd : seeds) {
    if (!sd) continue;
    if (int rc = check_same(acc0, sd, "rnt_keyswitch_ext")) return rc;
    if (!sd->in_ntt) return fail(RNT_ERR_DOMAIN_MISMATCH, "key-switch seeds must be in the NTT domain");
    if (sd->n_polys != acc0->n_polys) return fail(RNT_ERR_BAD_ARGUMENT, "key-switch seed batch differs");
  }
  if (acc0 == acc1) return fail(RNT_ERR_BAD_ARGUMENT, "rnt_keyswitch_ext: outputs alias");
  if (int rc = set_device(acc0->ctx)) return rc;
  rnt::Launch k = launch_for(acc0);
  const size_t Lt = k.L, Ls = src_limbs, n = k.t->n, wb = word_bytes(k.t), B = acc0->n_polys;
  const uint64_t src_ls = (uint64_t)B * n, full_ls = limb_stride(acc0);
  if (rnt::ks_whole_ok(k.t)) {
    // 2^10 <= N <= 2^14: the whole batch in one launch, no S
    rnt::Launch kw = k;
    kw.Ls = Ls;
    LAUNCH(kw.t, rnt::K_KS_WHOLE,
           rnt::launch_ks_whole(kw, acc0->data, acc1->data, full_ls, src, src_ls, key_a->data, key_b->data,
                                limb_stride(key_a), init0 ? init0->data : nullptr, init1 ? init1->data : nullptr,
                                full_ls, nullptr),
           "whole-plane key-switch");
    acc0->in_ntt = acc1->in_ntt = 0;
    return RNT_OK;
  }
  // polys per chunk: S is [Lt][Ls][Bc][N]
  size_t bc = std::max<size_t>(1, k.t->ks_ws_bytes / std::max<size_t>(1, Lt * Ls * n * wb));
  bc = std::min(bc, B);
  CallWs ws(acc0);
  if (int rc = ws.get((Lt * Ls + 2 * Lt) * bc * n * wb)) return rc;
  for (size_t p0 = 0; p0 < B; p0 += bc) {
    rnt::Launch kc = k;
    kc.B = std::min(bc, B - p0);
    kc.Ls = Ls;
    const uint64_t cls = (uint64_t)kc.B * n;
    char* S = (char*)ws.p;
    char* U0 = S + Lt * Ls * kc.B * n * wb;
    char* U1 = U0 + Lt * kc.B * n * wb;
    const size_t off = p0 * n * wb;
    const char* i0 = init0 ? (const char*)init0->data + off : nullptr;
    const char* i1 = init1 ? (const char*)init1->data + off : nullptr;
    if (int rc = ks_decompose_rows(kc, S, (const char*)src + off, src_ls, U0, U1, cls, key_a, key_b,
                                   i0, i1, full_ls))
      return rc;
    LAUNCH(kc.t, rnt::K_COL_INV,
           rnt::launch_col_inv(kc, (char*)acc0->data + off, full_ls, U0, cls, 1, nullptr), "ks inverse");
    LAUNCH(kc.t, rnt::K_COL_INV,
           rnt::launch_col_inv(kc, (char*)acc1->data + off, full_ls, U1, cls, 1, nullptr), "ks inverse");
  }
  acc0->in_ntt = acc1->in_ntt = 0;
  return RNT_OK;
}

extern "C" int rnt_ct_tensor(rnt_buf* d0, rnt_buf* d1, rnt_buf* d2, const rnt_buf* c0,
                             const rnt_buf* c1, const rnt_buf* c0p, const rnt_buf* c1p) {
  const rnt_buf* all[7] = {d0, d1, d2, c0, c1, c0p, c1p};
  for (const rnt_buf* b : all)
    if (int rc = check_buf(b, "rnt_ct_tensor")) return rc;
  for (int i = 1; i < 7; ++i)
    if (int rc = check_same(all[0], all[i], "rnt_ct_tensor")) return rc;
  if (c0->in_ntt || c1->in_ntt || c0p->in_ntt || c1p->in_ntt)
    return fail(RNT_ERR_DOMAIN_MISMATCH, "rnt_ct_tensor: inputs must be in coefficient domain");
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 7; ++j)
      if (i != j && all[i] == all[j])
        return fail(RNT_ERR_BAD_ARGUMENT, "rnt_ct_tensor: outputs must not alias other operands");
  if (int rc = set_device(c0->ctx)) return rc;
  rnt::Launch k = launch_for(c0);
  const size_t L = k.L, n = k.t->n, wb = word_bytes(k.t);
  const uint64_t ls = limb_stride(c0);
  if (rnt::tensor_whole_ok(k.t)) {
    LAUNCH(k.t, rnt::K_TENSOR_WHOLE,
           rnt::launch_tensor_whole(k, d0->data, d1->data, d2->data, ls, c0->data, c1->data, c0p->data, c1p->data, ls),
           "tensor whole");
    d0->in_ntt = d1->in_ntt = 1;
    d2->in_ntt = 0;
    return RNT_OK;
  }
  CallWs ws(d0);
  if (use_mf(k)) {  // N = 2^16, u32: the matrix-core tensor, one launch
    if (int rc = ws.get(rnt::plane_scratch_planes((uint64_t)L * c0->n_polys) * n * wb)) return rc;
    LAUNCH(k.t, rnt::K_MF_TENSOR,
           rnt::launch_mf_tensor(k, d0->data, d1->data, d2->data, ls, c0->data, c1->data, c0p->data, c1p->data,
                                 ls, ws.p),
           "MFMA tensor");
    d0->in_ntt = d1->in_ntt = 1;
    d2->in_ntt = 0;
    return RNT_OK;
  }
  if (int rc = ws.get(4 * L * c0->n_polys * n * wb)) return rc;
  char* T[4];
  for (int i = 0; i < 4; ++i) T[i] = (char*)ws.p + i * L * c0->n_polys * n * wb;
  LAUNCH(k.t, rnt::K_COL_FWD, rnt::launch_col_fwd(k, T[0], c0->data, T[1], c1->data, ls, ls), "tensor column");
  LAUNCH(k.t, rnt::K_COL_FWD, rnt::launch_col_fwd(k, T[2], c0p->data, T[3], c1p->data, ls, ls), "tensor column");
  LAUNCH(k.t, rnt::K_TENSOR_ROWS,
         rnt::launch_tensor_rows(k, d0->data, d1->data, d2->data, T[0], T[1], T[2], T[3], ls), "tensor rows");
  LAUNCH(k.t, rnt::K_COL_INV, rnt::launch_col_inv(k, d2->data, ls, d2->data, ls, 1, nullptr), "d2 inverse");
  d0->in_ntt = d1->in_ntt = 1;
  d2->in_ntt = 0;
  return RNT_OK;
}

// The ct-mul body; with `resc` the outputs are on drop_last(1) and each
// chunk's key-switch inverse applies the rescale as its epilogue
// (rnt_ct_mul_relin_rescale: the dropped limb's inverse runs first, into a
// chunk plane the other limbs' inverse reads), so the un-rescaled product
// never goes through HBM.
static int ct_mul_relin_body(rnt_buf* out0, rnt_buf* out1, const rnt_buf* c0, const rnt_buf* c1,
                             const rnt_buf* c0p, const rnt_buf* c1p, const rnt_buf* key_a,
                             const rnt_buf* key_b, bool resc) {
  if (int rc = set_device(c0->ctx)) return rc;
  rnt::Launch k = launch_for(c0);
  const size_t L = k.L, n = k.t->n, wb = word_bytes(k.t), B = c0->n_polys;
  const size_t bc = ks_chunk(k.t, L, B);
  // ws: [T0..T3 (column outputs, chunk-local)] | D0 | D1 | D2 | key-switch (S|U0|U1)
  // [| LAST0 | LAST1 with resc]
  // (the whole-plane tensor reads the ciphertexts directly: no T)
  const bool whole = rnt::tensor_whole_ok(k.t);
  const bool mf = !whole && use_mf(k);
  const size_t chunk_words = L * bc * n;
  // (the matrix-core tensor's scratch: plane_scratch_planes(L bc) <= L bc planes)
  const size_t nt = whole ? 0 : mf ? 1 : 4;
  // the key-switch's diagonal from the tensor's d2^ (one more chunk plane
  // set, D2H): the four-step key-switch on tiled grids, whose tensor writes it
  const bool diag = k.t->ks_diag && !whole && !rnt::ks_whole_ok(k.t) && rnt::col_resc_ok(k.t);
  const size_t need = ((nt + 3 + (diag ? 1 : 0)) * chunk_words + ks_scratch_words(k.t, L, bc) +
                       (resc ? 2 * bc * n : 0)) * wb;
  CallWs cws(out0);
  if (int rc = cws.get(need)) return rc;
  char* ws = (char*)cws.p;
  char* T[4];
  for (int i = 0; i < 4; ++i) T[i] = ws + i * chunk_words * wb;
  char* D0 = ws + nt * chunk_words * wb;
  char* D1 = D0 + chunk_words * wb;
  char* D2 = D1 + chunk_words * wb;
  char* KS = D2 + chunk_words * wb;
  char* D2H = nullptr;
  if (diag) {
    D2H = KS + ks_scratch_words(k.t, L, bc) * wb + (resc ? 2 * bc * n * wb : 0);
  }
  const uint64_t full_ls = limb_stride(c0);
  for (size_t p0 = 0; p0 < B; p0 += bc) {
    const size_t c = std::min(bc, B - p0);
    rnt::Launch kc = k;
    kc.B = c;
    const uint64_t cls = (uint64_t)c * n;
    if (diag) {
      kc.d2hat = D2H;  // written by the tensor, read by the key-switch rows
      kc.d2hat_ls = cls;
    }
    auto off = [&](const rnt_buf* b) { return (const char*)b->data + p0 * n * wb; };
    if (whole) {
      // d0^, d1^ NTT-resident and d2 in coefficient domain (engine.rs:486-493), one
      // launch reading the ciphertexts in place (full limb stride) into D0..D2 (chunk's)
      LAUNCH(kc.t, rnt::K_TENSOR_WHOLE,
             rnt::launch_tensor_whole(kc, D0, D1, D2, cls, off(c0), off(c1), off(c0p), off(c1p), full_ls),
             "tensor whole");
    } else if (mf) {
      // the same on the matrix-core transforms (N = 2^16), T0.. as its scratch
      LAUNCH(kc.t, rnt::K_MF_TENSOR,
             rnt::launch_mf_tensor(kc, D0, D1, D2, cls, off(c0), off(c1), off(c0p), off(c1p), full_ls, T[0]),
             "MFMA tensor");
    } else {
    LAUNCH(kc.t, rnt::K_COL_FWD, rnt::launch_col_fwd(kc, T[0], off(c0), T[1], off(c1), full_ls, cls), "tensor column");
    LAUNCH(kc.t, rnt::K_COL_FWD, rnt::launch_col_fwd(kc, T[2], off(c0p), T[3], off(c1p), full_ls, cls), "tensor column");
    LAUNCH(kc.t, rnt::K_TENSOR_ROWS, rnt::launch_tensor_rows(kc, D0, D1, D2, T[0], T[1], T[2], T[3], cls), "tensor rows");
    // d2 -> coefficient domain (engine.rs:493), in place in D2
    LAUNCH(kc.t, rnt::K_COL_INV, rnt::launch_col_inv(kc, D2, cls, D2, cls, 1, nullptr), "d2 inverse");
    }
    if (resc) {
      // gadget sum into the chunk's NTT-row accumulators, then the inverse
      // with the rescale fused (engine.rs:263-282 after :530-531)
      char* S = KS;
      char* U0 = S + L * L * c * n * wb;
      char* U1 = U0 + L * c * n * wb;
      char* LAST0 = KS + ks_scratch_words(k.t, L, bc) * wb;
      char* LAST1 = LAST0 + bc * n * wb;
      if (int rc = ks_decompose_rows(kc, S, D2, cls, U0, U1, cls, key_a, key_b, D0, D1, cls)) return rc;
      rnt::Launch kl = kc;  // the dropped limb: its coefficient plane only
      kl.L = 1;
      rnt::ColRescArgs la;
      la.limb0 = (uint32_t)(L - 1);
      rnt::Launch kr = kc;  // the kept limbs, rescaled by it
      kr.L = L - 1;
      const uint64_t rls = limb_stride(out0);
      char* U[2] = {U0, U1};
      char* LAST[2] = {LAST0, LAST1};
      rnt_buf* O[2] = {out0, out1};
      for (int o = 0; o < 2; ++o) {
        LAUNCH(kl.t, rnt::K_COL_INV,
               rnt::launch_col_inv(kl, LAST[o], cls, U[o] + (L - 1) * cls * wb, cls, 1, nullptr, false, la),
               "ks inverse (dropped limb)");
        rnt::ColRescArgs ra;
        ra.last = LAST[o];
        ra.inv = rnt::resc_inv_row(k.t, L - 1, 0);
        ra.invp = rnt::resc_inv_row(k.t, L - 1, 1);
        LAUNCH(kr.t, rnt::K_COL_INV,
               rnt::launch_col_inv(kr, (char*)O[o]->data + p0 * n * wb, rls, U[o], cls, 1, nullptr, false, ra),
               "ks inverse + rescale");
      }
      continue;
    }
    // gadget sum with d0hat / d1hat as accumulator seeds (engine.rs:530-531)
    // d2 lives in a chunk-local buffer: present it as a full "buffer".
    rnt_buf d2view;
    d2view.ctx = c0->ctx;
    d2view.n_polys = c;
    d2view.data = D2;
    if (int rc = ks_chunk_run(kc, KS, &d2view, 0, c, key_a, key_b, (char*)out0->data + p0 * n * wb,
                              (char*)out1->data + p0 * n * wb, full_ls, D0, D1, cls, nullptr, 1))
      return rc;
    d2view.data = nullptr;  // not owned
  }
  out0->in_ntt = out1->in_ntt = 0;
  return RNT_OK;
}

static int ct_mul_check(rnt_buf* out0, rnt_buf* out1, const rnt_buf* c0, const rnt_buf* c1,
                        const rnt_buf* c0p, const rnt_buf* c1p, const rnt_buf* key_a, const rnt_buf* key_b,
                        const char* name) {
  const rnt_buf* all[6] = {out0, out1, c0, c1, c0p, c1p};
  for (const rnt_buf* b : all)
    if (int rc = check_buf(b, name)) return rc;
  for (int i = 3; i < 6; ++i)
    if (int rc = check_same(c0, all[i], name)) return rc;
  if (int rc = check_key(c0, key_a, key_b)) return rc;
  if (c0->in_ntt || c1->in_ntt || c0p->in_ntt || c1p->in_ntt)
    return fail(RNT_ERR_DOMAIN_MISMATCH, "mul_ciphertexts_gadget: inputs must be in coefficient domain");
  if (out0 == out1) return fail(RNT_ERR_BAD_ARGUMENT, "%s: out0 aliases out1", name);
  return RNT_OK;
}

extern "C" int rnt_ct_mul_relin(rnt_buf* out0, rnt_buf* out1, const rnt_buf* c0,
                                const rnt_buf* c1, const rnt_buf* c0p, const rnt_buf* c1p,
                                const rnt_buf* key_a, const rnt_buf* key_b) {
  if (int rc = ct_mul_check(out0, out1, c0, c1, c0p, c1p, key_a, key_b, "rnt_ct_mul_relin")) return rc;
  if (int rc = check_same(out0, c0, "rnt_ct_mul_relin")) return rc;
  if (int rc = check_same(out1, c0, "rnt_ct_mul_relin")) return rc;
  return ct_mul_relin_body(out0, out1, c0, c1, c0p, c1p, key_a, key_b, false);
}

extern "C" int rnt_ct_mul_relin_rescale(rnt_buf* out0, rnt_buf* out1, const rnt_buf* c0,
                                        const rnt_buf* c1, const rnt_buf* c0p, const rnt_buf* c1p,
                                        const rnt_buf* key_a, const rnt_buf* key_b) {
  if (int rc = ct_mul_check(out0, out1, c0, c1, c0p, c1p, key_a, key_b, "rnt_ct_mul_relin_rescale")) return rc;
  const size_t L = c0->ctx->L;
  if (L < 2)  // poly.rs:191-197
    return fail_fields(RNT_ERR_INVALID_MOD_DROP, 1, L, "invalid mod-drop count 1 for %zu channels", L);
  for (const rnt_buf* o : {(const rnt_buf*)out0, (const rnt_buf*)out1}) {
    if (o->ctx->t != c0->ctx->t || o->ctx->L != L - 1)
      return fail(RNT_ERR_BASIS_MISMATCH, "rescale: output basis is not drop_last(1) of the input's");
    if (o->n_polys != c0->n_polys) return fail(RNT_ERR_BAD_ARGUMENT, "rescale: batch sizes differ");
  }
  if (out0->ctx != out1->ctx)  // engine.rs:272-274: one shared new basis
    return fail(RNT_ERR_BASIS_MISMATCH, "rescale_ciphertext: outputs must share one basis");
  if (rnt::col_resc_ok(c0->ctx->t.get()) && !rnt::ks_whole_ok(c0->ctx->t.get()))
    return ct_mul_relin_body(out0, out1, c0, c1, c0p, c1p, key_a, key_b, true);
  // small rings (the whole-plane key-switch, no column inverse): the product,
  // then the rescale, through two call-scoped temporaries
  rnt_buf* t0 = nullptr;
  rnt_buf* t1 = nullptr;
  int rc = rnt_buf_alloc_uninit(c0->ctx, c0->n_polys, &t0);
  if (rc == RNT_OK) rc = rnt_buf_alloc_uninit(c0->ctx, c0->n_polys, &t1);
  if (rc == RNT_OK) rc = ct_mul_relin_body(t0, t1, c0, c1, c0p, c1p, key_a, key_b, false);
  if (rc == RNT_OK) rc = rnt_ct_rescale(out0, out1, t0, t1);
  rnt_buf_free(t0);
  rnt_buf_free(t1);
  return rc;
}

extern "C" int rnt_ct_rotate(rnt_buf* out0, rnt_buf* out1, const rnt_buf* c0, const rnt_buf* c1,
                             int32_t kk, const rnt_buf* key_a, const rnt_buf* key_b) {
  const rnt_buf* all[4] = {out0, out1, c0, c1};
  for (const rnt_buf* b : all)
    if (int rc = check_buf(b, "rnt_ct_rotate")) return rc;
  for (int i = 1; i < 4; ++i)
    if (int rc = check_same(all[0], all[i], "rnt_ct_rotate")) return rc;
  if (int rc = check_key(c0, key_a, key_b)) return rc;
  if (out0 == out1) return fail(RNT_ERR_BAD_ARGUMENT, "rnt_ct_rotate: out0 aliases out1");
  if (int rc = set_device(c0->ctx)) return rc;
  rnt::Launch k = launch_for(c0);
  const size_t L = k.L, n = k.t->n, wb = word_bytes(k.t), B = c0->n_polys;
  const size_t words = L * B * n;
  const uint64_t g = rotation_exponent(kk, 2 * (uint64_t)n);
  // ws: SIG0 | SIG1 | [TMP when an input is NTT-domain] | key-switch chunk space
  const size_t bc = ks_chunk(k.t, L, B);
  const bool any_ntt = c0->in_ntt || c1->in_ntt;
  // sigma(c0) needs no launch of its own on the tiled four-step key-switch:
  // its inverse column pass gathers it from c0 as it adds it (k_colt_inv's
  // addend with g^-1 mod 2N).  Only for one ciphertext by default
  // (RNT_ROT_FUSE=1; 2: any batch, 0: never): the scattered 4-byte gather
  // costs the inverse about what the automorphism launch costs, which at one
  // ciphertext is mostly launch and tail (config 5: +2.0% at one ciphertext,
  // -0.5% at eight, profiles/r06/ab_rot_fuse.txt).  Not in place on out0: a
  // workgroup's gather would race the stores of the others on the same plane
  const bool fuse0 = (k.t->rot_fuse == 2 || (k.t->rot_fuse == 1 && B == 1)) && (g & 1) && !c0->in_ntt &&
                     !rnt::ks_whole_ok(k.t) && rnt::col_resc_ok(k.t) && out0->data != c0->data;
  const size_t tmp_words = any_ntt ? words : 0;
  CallWs ws(out0);
  if (int rc = ws.get((2 * words + tmp_words + ks_scratch_words(k.t, L, bc)) * wb)) return rc;
  char* sig0 = (char*)ws.p;
  char* sig1 = sig0 + words * wb;
  char* tmp = sig1 + words * wb;
  char* KS = tmp + tmp_words * wb;
  // sigma(c0), sigma(c1) in coefficient domain (engine.rs:417-419; poly.rs:494-504
  // converts an NTT-domain input first)
  for (int i = fuse0 ? 1 : 0; i < 2; ++i) {
    const rnt_buf* src = i ? c1 : c0;
    char* dst = i ? sig1 : sig0;
    const void* s = src->data;
    if (src->in_ntt) {
      if (int rc = to_coeff_into(src, tmp)) return rc;
      s = tmp;
    }
    LAUNCH(k.t, rnt::K_AUTOMORPHISM, rnt::launch_automorphism(k, dst, s, g), "automorphism");
  }
  rnt_buf sview;
  sview.ctx = c0->ctx;
  sview.n_polys = B;
  sview.data = sig1;
  const uint64_t ls = limb_stride(c0);
  rnt::Launch kr = k;
  if (fuse0) {
    // g^-1 mod 2N (g odd): Newton's iteration mod 2^64, then the mask
    uint64_t x = g;
    for (int it = 0; it < 6; ++it) x *= 2 - g * x;
    kr.add_ginv = (uint32_t)(x & (2 * (uint64_t)n - 1));
  }
  for (size_t p0 = 0; p0 < B; p0 += bc) {
    const size_t c = std::min(bc, B - p0);
    if (int rc = ks_chunk_run(kr, KS, &sview, p0, c, key_a, key_b, out0->data, out1->data, ls,
                              nullptr, nullptr, 0, fuse0 ? c0->data : sig0, 0))
      return rc;
  }
  sview.data = nullptr;
  out0->in_ntt = out1->in_ntt = 0;
  return RNT_OK;
}

extern "C" int rnt_ct_rescale(rnt_buf* out0, rnt_buf* out1, const rnt_buf* c0, const rnt_buf* c1) {
  if (int rc = check_buf(out0, "rnt_ct_rescale")) return rc;
  if (int rc = check_buf(out1, "rnt_ct_rescale")) return rc;
  if (out0->ctx != out1->ctx)  // engine.rs:272-274: one shared new basis
    return fail(RNT_ERR_BASIS_MISMATCH, "rescale_ciphertext: outputs must share one basis");
  if (int rc = rnt_rescale(out0, c0)) return rc;
  return rnt_rescale(out1, c1);
}

// ---------------------------------------------------------------------------
// device count / profiling
// ---------------------------------------------------------------------------
extern "C" int rnt_device_count(int* n) {
  if (!n) return fail(RNT_ERR_BAD_ARGUMENT, "null out");
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  *n = c;
  return RNT_OK;
}

extern "C" int rnt_profile_enable(const rnt_ctx* ctx, int enable) {
  if (!ctx) return fail(RNT_ERR_BAD_ARGUMENT, "null ctx");
  rnt::Tables* t = ctx->t.get();
  if (int rc = set_device(ctx)) return rc;
  HIP_TRY(hipStreamSynchronize(t->stream), "hipStreamSynchronize");
  if (t->prof == nullptr) {
    try {
      t->prof = new rnt::Prof;
    } catch (...) {
      return fail(RNT_ERR_OUT_OF_MEMORY, "host allocation failed");
    }
  }
  std::lock_guard<std::mutex> g(t->prof->mu);
  for (auto& r : t->prof->pending) {
    t->prof->pool.push_back(r.a);
    t->prof->pool.push_back(r.b);
  }
  t->prof->pending.clear();
  for (int i = 0; i < rnt::K_COUNT; ++i) {
    t->prof->launches[i] = 0;
    t->prof->ms[i] = 0;
  }
  t->prof->on = enable != 0;
  return RNT_OK;
}

extern "C" int rnt_profile_read(const rnt_ctx* ctx, const char* kernel, uint64_t* launches,
                                double* total_ms) {
  if (!ctx || !kernel || !launches || !total_ms) return fail(RNT_ERR_BAD_ARGUMENT, "null argument");
  rnt::Tables* t = ctx->t.get();
  int id = -1;
  for (int i = 0; i < rnt::K_COUNT; ++i)
    if (std::strcmp(kKernelNames[i], kernel) == 0) id = i;
  if (id < 0) return fail(RNT_ERR_BAD_ARGUMENT, "unknown kernel name '%s'", kernel);
  *launches = 0;
  *total_ms = 0;
  if (t->prof == nullptr) return RNT_OK;
  if (int rc = set_device(ctx)) return rc;
  HIP_TRY(hipStreamSynchronize(t->stream), "hipStreamSynchronize");
  std::lock_guard<std::mutex> g(t->prof->mu);
  for (auto& r : t->prof->pending) {
    float ms = 0;
    if (const hipError_t e = hipEventElapsedTime(&ms, r.a, r.b); e == hipSuccess) {
      t->prof->launches[r.id] += 1;
      t->prof->ms[r.id] += ms;
    } else {
      prof_fail(t->prof, e, "hipEventElapsedTime(profile)");
    }
    t->prof->pool.push_back(r.a);
    t->prof->pool.push_back(r.b);
  }
  t->prof->pending.clear();
  *launches = t->prof->launches[id];
  *total_ms = t->prof->ms[id];
  if (t->prof->err != hipSuccess) {
    const hipError_t e = t->prof->err;
    const char* where = t->prof->err_where;
    t->prof->err = hipSuccess;
    return fail(RNT_ERR_DEVICE, "%s failed: %s (profiling was turned off; the launches ran)", where,
                hipGetErrorString(e));
  }
  return RNT_OK;
}
