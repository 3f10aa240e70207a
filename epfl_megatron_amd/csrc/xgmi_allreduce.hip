// One-shot all-reduce / all-gather over xGMI peer memory for small,
// latency-bound messages
// (the TP all-reduces of a decode step are [b, h] = a few KiB,
// where a ring collective's 2(W-1) link hops and its launch / proxy overhead
// dominate).  RCCL stays the default and the fallback (parallel/comm.py routes
// here only for registered groups and messages within the registered capacity).
//
// Each rank owns one uncached device region (hipExtMallocWithFlags
// hipDeviceMallocUncached: no L2 line of it is ever stale, so peers need no
// cache maintenance) exported with an IPC handle and mapped by every peer:
//
//   data   [2 parity][W source slots][cap bytes]   written by the peers
//   flags  [MAXWG][W]  u32                          written by the peers
//   epoch  [MAXWG]     u32                          this rank only
//   error  u32                                      this rank only
//
// Push form, one launch per call: workgroup b owns the fixed 4 KiB chunk b of
// the message; it stores its chunk into slot `rank` of every peer's region
// (W-1 remote xGMI writes, posted), publishes "chunk b of epoch e is there" in
// each peer's flags[b][rank], waits until every peer published the same for
// its region, then sums the W slots from its own (local) memory in rank order
// (every rank adds in the same order: the results are bitwise equal across the
// group, as TP replicas require).  No grid-wide barrier: a chunk's data and
// its flags travel together per workgroup.  Two parities make one barrier per
// call enough: a peer can run at most one call ahead (it needs our arrival for
// epoch e before it reaches e+1), and e+1 writes the other parity.  Epochs are
// device-side per workgroup, so the launch is hipGraph-capturable.
//
// Ordering (MI355X_MICROARCH "Valid forms", system scope because the peers
// are other GPUs): every storing wave drains its stores (s_waitcnt vmcnt(0)),
// the workgroup barrier, then the flag lanes issue a system-scope RELEASE fence,
// wait for it (asm vmcnt(0): ROCm 7.2 can drop the fence's own wait) and store
// the flag relaxed; the polling lanes poll relaxed, then issue ONE system-scope
// ACQUIRE fence and its wait before the barrier that releases the readers.
//
// The waits are bounded by wall clock (s_memrealtime, 100 MHz; timeout_ms,
// default 1 s, EMA_XGMI_TIMEOUT_MS): on timeout the error word is set, the
// workgroup's output chunk is filled with NaN (never stale partial sums that
// look valid) and the kernel ends instead of hanging the GPU on a dead peer;
// XgmiAllReduce.check() raises on the error word, and the training log and
// every generate call check it.
#include "common.h"
#include "kernels.h"

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace ema {
namespace {

constexpr int XG_THREADS = 256;
constexpr int64_t XG_CHUNK = XG_THREADS * 16;  // bytes per workgroup
constexpr int XG_MAXW = 8;

struct XgArgs {
  char* data[XG_MAXW];       // peer p's data region (p == rank: own)
  unsigned* flags[XG_MAXW];  // peer p's flags
  unsigned* own_flags;
  unsigned* epoch;
  unsigned* error;
  const char* in;
  char* out;
  int64_t nbytes, cap;
  uint64_t timeout_ticks;  // s_memrealtime ticks (100 MHz)
  int rank, world;
};

// GATHER: out[p * nbytes + off] = rank p's chunk (all-gather along dim 0)
// instead of the rank-ordered sum; same transport, flags and parities.
template <typename T, bool GATHER>
__global__ __launch_bounds__(XG_THREADS) void xgmi_oneshot_k(const XgArgs a) {
  const int b = blockIdx.x, t = threadIdx.x;
  const int64_t off = (int64_t)b * XG_CHUNK + (int64_t)t * 16;
  const bool valid = off < a.nbytes;
  const unsigned e = a.epoch[b] + 1u;
  const int64_t par = (int64_t)(e & 1u) * a.world * a.cap;
  __shared__ int timed_out;
  if (t == 0) timed_out = 0;
  V16<T> v;
  if (valid) {
    v = ld16(reinterpret_cast<const T*>(a.in + off));
    for (int p = 0; p < a.world; ++p)
      st16(reinterpret_cast<T*>(a.data[p] + par + (int64_t)a.rank * a.cap + off), v);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's slot stores done
  __syncthreads();                                   // ... and every wave's
  if (t < a.world) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");     // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(a.flags[t] + (int64_t)b * a.world + a.rank, e, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned* f = a.own_flags + (int64_t)b * a.world + t;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    // (a peer may already be one epoch ahead: >= in wrap-safe form)
    while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
        __hip_atomic_store(a.error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        timed_out = 1;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");     // system scope, once per lane
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (timed_out) {  // a peer never arrived: poison this chunk of the output
    if (valid) {
      V16<T> nan;
#pragma unroll
      for (int i = 0; i < V16<T>::N; ++i) nan.v[i] = from_f<T>(__builtin_nanf(""));
      const int reps = GATHER ? a.world : 1;
      for (int p = 0; p < reps; ++p) st16(reinterpret_cast<T*>(a.out + (int64_t)p * a.nbytes + off), nan);
    }
    if (t == 0) a.epoch[b] = e;
    return;
  }
  if (GATHER) {
    if (valid)
      for (int p = 0; p < a.world; ++p)
        st16(reinterpret_cast<T*>(a.out + (int64_t)p * a.nbytes + off),
             ld16(reinterpret_cast<const T*>(a.data[a.rank] + par + (int64_t)p * a.cap + off)));
  } else if (valid) {
    constexpr int N = V16<T>::N;
    float acc[N];
#pragma unroll
    for (int i = 0; i < N; ++i) acc[i] = 0.f;
    for (int p = 0; p < a.world; ++p) {
      const V16<T> x = ld16(reinterpret_cast<const T*>(a.data[a.rank] + par + (int64_t)p * a.cap + off));
#pragma unroll
      for (int i = 0; i < N; ++i) acc[i] += to_f(x.v[i]);
    }
    V16<T> o;
#pragma unroll
    for (int i = 0; i < N; ++i) o.v[i] = from_f<T>(acc[i]);
    st16(reinterpret_cast<T*>(a.out + off), o);
  }
  if (t == 0) a.epoch[b] = e;
}

// Wall-clock bound of a peer wait (ms).  Long by default: TP ranks drift apart
// through host work (a checkpoint write, first-iteration setup, a GC pause),
// and a healthy-but-late peer must never trip it.  A latency-
// critical caller (decode serving) may set a short bound per communicator
// (xgmi_set_timeout); EMA_XGMI_TIMEOUT_MS overrides the default.
int64_t default_timeout_ms() {
  static const int64_t ms = [] {
    const char* e = getenv("EMA_XGMI_TIMEOUT_MS");
    const long v = e ? atol(e) : 0;
    return (int64_t)(v > 0 ? v : 60000);
  }();
  return ms;
}

struct XgComm {
  int rank = 0, world = 0, dev = 0;
  int64_t cap = 0, maxwg = 0;
  int64_t timeout_ms = 0;           // peer-wait bound (default_timeout_ms())
  char* base = nullptr;             // own region
  std::vector<char*> peers;         // mapped peer regions (own at [rank])
  int64_t data_bytes() const { return 2 * (int64_t)world * cap; }
  int64_t flags_off() const { return data_bytes(); }
  int64_t epoch_off() const { return flags_off() + maxwg * world * 4; }
  int64_t error_off() const { return epoch_off() + maxwg * 4; }
  int64_t total() const { return error_off() + 256; }
};

std::mutex g_mu;
std::vector<XgComm*> g_comms;

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("xgmi: ") + what + ": " + hipGetErrorString(e));
}

XgComm* get(int64_t id) {
  std::lock_guard<std::mutex> l(g_mu);
  if (id < 0 || id >= (int64_t)g_comms.size() || !g_comms[id]) throw std::runtime_error("xgmi: bad id");
  return g_comms[id];
}

}  // namespace

int64_t xgmi_create(int rank, int world, int64_t cap, void* handle_out) {
  if (world < 2 || world > XG_MAXW || rank < 0 || rank >= world)
    throw std::runtime_error("xgmi: world must be 2..8");
  if (cap <= 0 || cap % XG_CHUNK) throw std::runtime_error("xgmi: cap must be a multiple of 4 KiB");
  auto* c = new XgComm();
  c->rank = rank;
  c->world = world;
  c->cap = cap;
  c->maxwg = cap / XG_CHUNK;
  c->timeout_ms = default_timeout_ms();
  hip_ok(hipGetDevice(&c->dev), "hipGetDevice");
  void* p = nullptr;
  hip_ok(hipExtMallocWithFlags(&p, (size_t)c->total(), hipDeviceMallocUncached), "uncached malloc");
  c->base = static_cast<char*>(p);
  hip_ok(hipMemset(c->base, 0, (size_t)c->total()), "memset");
  hip_ok(hipDeviceSynchronize(), "sync");
  hipIpcMemHandle_t h;
  hip_ok(hipIpcGetMemHandle(&h, c->base), "hipIpcGetMemHandle");
  std::memcpy(handle_out, &h, sizeof(h));
  c->peers.assign(world, nullptr);
  c->peers[rank] = c->base;
  std::lock_guard<std::mutex> l(g_mu);
  g_comms.push_back(c);
  return (int64_t)g_comms.size() - 1;
}

int xgmi_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

void xgmi_open(int64_t id, const void* handles) {
  XgComm* c = get(id);
  for (int p = 0; p < c->world; ++p) {
    if (p == c->rank) continue;
    hipIpcMemHandle_t h;
    std::memcpy(&h, static_cast<const char*>(handles) + (size_t)p * sizeof(h), sizeof(h));
    void* q = nullptr;
    hip_ok(hipIpcOpenMemHandle(&q, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    c->peers[p] = static_cast<char*>(q);
  }
}

int64_t xgmi_capacity(int64_t id) { return get(id)->cap; }


void xgmi_launch(int64_t id, const void* in, void* out, int64_t nbytes, int dt, bool gather,
                 hipStream_t s) {
  XgComm* c = get(id);
  if (nbytes <= 0) return;
  if (nbytes > c->cap || nbytes % 16) throw std::runtime_error("xgmi: message exceeds capacity or is not 16-B sized");
  for (int p = 0; p < c->world; ++p)
    if (!c->peers[p]) throw std::runtime_error("xgmi: peers not opened");
  XgArgs a{};
  for (int p = 0; p < c->world; ++p) {
    a.data[p] = c->peers[p];
    a.flags[p] = reinterpret_cast<unsigned*>(c->peers[p] + c->flags_off());
  }
  a.own_flags = reinterpret_cast<unsigned*>(c->base + c->flags_off());
  a.epoch = reinterpret_cast<unsigned*>(c->base + c->epoch_off());
  a.error = reinterpret_cast<unsigned*>(c->base + c->error_off());
  a.in = static_cast<const char*>(in);
  a.out = static_cast<char*>(out);
  a.nbytes = nbytes;
  a.cap = c->cap;
  a.rank = c->rank;
  a.world = c->world;
  a.timeout_ticks = (uint64_t)c->timeout_ms * 100000ull;  // s_memrealtime runs at 100 MHz
  if ((uintptr_t)in % 16 || (uintptr_t)out % 16)
    throw std::runtime_error("xgmi: input and output must be 16-B aligned (parallel/xgmi.py stages)");
  const unsigned grid = (unsigned)((nbytes + XG_CHUNK - 1) / XG_CHUNK);
  if (gather) {
    EMA_DISPATCH_FLOAT(dt, T, {
      hipLaunchKernelGGL((xgmi_oneshot_k<T, true>), dim3(grid), dim3(XG_THREADS), 0, s, a);
    });
  } else {
    EMA_DISPATCH_FLOAT(dt, T, {
      hipLaunchKernelGGL((xgmi_oneshot_k<T, false>), dim3(grid), dim3(XG_THREADS), 0, s, a);
    });
  }
}

void xgmi_all_reduce(int64_t id, const void* in, void* out, int64_t nbytes, int dt, hipStream_t s) {
  xgmi_launch(id, in, out, nbytes, dt, false, s);
}

void xgmi_all_gather(int64_t id, const void* in, void* out, int64_t nbytes, int dt, hipStream_t s) {
  xgmi_launch(id, in, out, nbytes, dt, true, s);
}

void xgmi_set_timeout(int64_t id, int64_t ms) {
  if (ms <= 0) throw std::runtime_error("xgmi: timeout must be positive");
  get(id)->timeout_ms = ms;
}

int64_t xgmi_get_timeout(int64_t id) { return get(id)->timeout_ms; }

void* xgmi_error_word(int64_t id) {
  XgComm* c = get(id);
  return c->base + c->error_off();
}

int xgmi_error(int64_t id) {
  XgComm* c = get(id);
  unsigned v = 0;
  hip_ok(hipMemcpy(&v, c->base + c->error_off(), 4, hipMemcpyDeviceToHost), "read error word");
  return (int)v;
}

void xgmi_destroy(int64_t id) {
  XgComm* c;
  {
    std::lock_guard<std::mutex> l(g_mu);
    if (id < 0 || id >= (int64_t)g_comms.size() || !g_comms[id]) return;
    c = g_comms[id];
    g_comms[id] = nullptr;
  }
  hipDeviceSynchronize();
  for (int p = 0; p < c->world; ++p)
    if (p != c->rank && c->peers[p]) hipIpcCloseMemHandle(c->peers[p]);
  hipFree(c->base);
  delete c;
}

}  // namespace ema
