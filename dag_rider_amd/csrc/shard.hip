// shard.hip -- process-column sharded reachability (include/dagrider_shard.h).
//
// for a DAG split across the GPUs of one node, GPU g keeps the
// target columns [g*C, (g+1)*C) of every strong row and the weak edges whose
// target falls there.  A batch of up to 64 queries sweeps the rounds top-down;
// the frontier of a round is held TRANSPOSED: FT[s] = u64 mask of the queries
// that reached source s (so one all-gather of C words per shard per round moves
// the frontier of all 64 queries).  Per round, one launch of k_shard_round:
//
//   1. write round r's reach rows (the ballot of bit b over 64 sources is query
//      b's bitset word -- a 64x64 bit transpose per wave, shard 0 only);
//   2. strong expansion into the pending frontier of r-1: each wave takes 64
//      sources; for every (source with a non-empty mask) x (row word) it walks
//      the active sources with a scalar loop (readlane) and lane j ORs the
//      source's query mask when the row has target bit j: one atomic per target;
//   3. weak expansion: the shard's weak edges of round r (sorted by (delta,
//      target)) OR the source's mask into the pending frontier of r - delta
//      (wave-uniform destinations collapse to one reduction + one atomic);
//   4. the last workgroup of the shard (threadfence + counter) drains the
//      pending frontier of r-1, adds queries that start there, and writes its
//      columns of FT_{r-1}: straight into the shared frontier buffer (local
//      mode) or into the send buffer of ncclAllGather (RCCL mode).
//
// Semantics are those of dr_reach_sets / dr_path_batch (process.go:89-148): the
// reach set is defined over the id space (a dangling target counts as reached,
// :123,136), an absent vertex has an all-zero row (no edges, :111-116), and the
// start vertex is in its own set (self path, :91-93).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "dagrider_gpu.h"
#include "dagrider_shard.h"

namespace {

typedef unsigned long long u64;
constexpr int SH_NT = 256;  // threads per workgroup (4 waves)
constexpr int SH_BATCH = 64;

thread_local std::string g_shard_err;

struct SBuf {
  void *p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t c = std::max<size_t>(bytes, 4096);
    hipError_t e = hipMalloc(&p, c);
    if (e == hipSuccess) cap = c;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T> T *as() const { return static_cast<T *>(p); }
};

struct QInfo {
  int32_t top, bottom, src0, pad;  // src0 = 0-based source of `from`, -1 none
  int64_t obase;                   // word offset of round `bottom` in the batch output
};

struct ShardArgs {
  const u64 *strong;        // [nlocal][max_rounds][n][WSs]
  const uint32_t *weak;     // per local shard: edges (target col 0-10, source 11-21, delta 22-31)
  const uint64_t *woff;     // [nlocal][max_rounds+1] edge offsets (absolute in weak)
  const u64 *ft;            // FT_r: [G*C] query masks
  u64 *ftn;                 // FT_{r-1} destination: full buffer (local) or send buffer (RCCL)
  u64 *pend;                // [nlocal][depth][C]
  unsigned *cnt;            // [nlocal] workgroups done this round
  u64 *out;                 // batch reach rows
  const QInfo *q;           // [nq]
  int32_t n, W, WSs, C, depth, shard0, local, max_rounds, nq, strong_only;
  int64_t strong_shard_stride;  // words per local shard of strong
};

__device__ __forceinline__ u64 shfl_xor64(u64 v, int m) {
  const int lo = __shfl_xor((int)(uint32_t)v, m, 64), hi = __shfl_xor((int)(uint32_t)(v >> 32), m, 64);
  return ((u64)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ u64 rdlane64(u64 x, int l) {
  return ((u64)(uint32_t)__builtin_amdgcn_readlane((int)(x >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
}

// round r of a batch sweep; see the file comment for the four steps.
__global__ void __launch_bounds__(SH_NT) k_shard_round(ShardArgs a, int r, u64 expmask, u64 outmask, u64 injmask,
                                                        int produce) {
  const int l = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int nwv = gridDim.x * (SH_NT / 64);
  const int gw = blockIdx.x * (SH_NT / 64) + (threadIdx.x >> 6);
  const int C = a.C;
  u64 *pend = a.pend + (size_t)l * a.depth * C;

  // 1 + 2: reach rows of round r and strong expansion into round r-1.  A wave's
  // work item is (64-source chunk, target word): nchunks * WSs items spread over
  // every wave of the grid; the chunk's first word also writes the reach rows.
  const int nchunks = (a.n + 63) >> 6;
  for (int it = gw; it < nchunks * a.WSs; it += nwv) {
    const int s0 = (it / a.WSs) * 64, tw = it % a.WSs;
    const int s = s0 + lane;
    const u64 m = s < a.n ? a.ft[s] : 0ULL;
    if (l == 0 && tw == 0 && outmask) {
      u64 mine = 0;
      for (u64 om = outmask; om; om &= om - 1) {
        const int b = __builtin_ctzll(om);
        const u64 word = __ballot((m >> b) & 1ULL);
        if (lane == b) mine = word;
      }
      if ((outmask >> lane) & 1ULL) {
        const QInfo qi = a.q[lane];
        a.out[qi.obase + (int64_t)(r - qi.bottom) * a.W + (s0 >> 6)] = mine;
      }
    }
    const u64 me = m & expmask;
    if (r < 1 || __ballot(me != 0ULL) == 0ULL) continue;
    const u64 row = (me != 0ULL)
                        ? a.strong[(size_t)l * a.strong_shard_stride + ((size_t)r * a.n + s) * a.WSs + tw]
                        : 0ULL;
    u64 act = __ballot(row != 0ULL);
    u64 acc = 0;
    while (act) {  // wave-uniform loop over the sources that contribute
      const int src = __builtin_ctzll(act);
      act &= act - 1;
      const u64 rs = rdlane64(row, src), ms = rdlane64(me, src);
      if ((rs >> lane) & 1ULL) acc |= ms;
    }
    if (acc) atomicOr(&pend[(size_t)((r - 1) & (a.depth - 1)) * C + tw * 64 + lane], acc);
  }

  // 3: weak expansion
  if (!a.strong_only && r >= 2) {
    const size_t e0 = a.woff[(size_t)l * (a.max_rounds + 1) + r], e1 = a.woff[(size_t)l * (a.max_rounds + 1) + r + 1];
    for (size_t base = e0 + (size_t)gw * 64; base < e1; base += (size_t)nwv * 64) {
      const size_t e = base + lane;
      u64 m = 0;
      uint32_t key = 0xFFFFFFFFu;
      if (e < e1) {
        const uint32_t w = a.weak[e];
        m = a.ft[(w >> 11) & 2047u] & expmask;
        const int slot = (r - (int)(w >> 22)) & (a.depth - 1);
        key = (uint32_t)slot * (uint32_t)C + (w & 2047u);
      }
      const u64 act = __ballot(m != 0ULL);
      if (!act) continue;
      const int first = __builtin_ctzll(act);
      const uint32_t kf = (uint32_t)__builtin_amdgcn_readlane((int)key, first);
      if (__ballot(m != 0ULL && key != kf) == 0ULL) {
        u64 v = m;
        for (int d = 32; d; d >>= 1) v |= shfl_xor64(v, d);
        if (lane == first) atomicOr(&pend[kf], v);
      } else if (m) {
        atomicOr(&pend[key], m);
      }
    }
  }

  // 4: the last workgroup of this shard produces its columns of FT_{r-1}
  if (!produce) return;
  __shared__ int last;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    last = atomicAdd(&a.cnt[l], 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  const int g = a.shard0 + l;
  u64 *slotp = pend + (size_t)((r - 1) & (a.depth - 1)) * C;
  for (int t = threadIdx.x; t < C; t += SH_NT) {
    u64 v = atomicExch(&slotp[t], 0ULL);
    const int col = g * C + t;
    for (u64 im = injmask; im; im &= im - 1) {
      const int b = __builtin_ctzll(im);
      if (a.q[b].src0 == col) v |= 1ULL << b;
    }
    a.ftn[(a.local ? (size_t)g * C : 0) + t] = v;
  }
  if (threadIdx.x == 0) a.cnt[l] = 0;
}

}  // namespace

struct dr_shard {
  int n = 0, f = 0, W = 0, G = 1, shard0 = 0, nlocal = 1, WSs = 1, C = 64, max_rounds = 0, dev = 0;
  bool local = true;
  int nrounds = 0, dmax = 1, depth = 2;
  size_t max_weak_round = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  ncclComm_t comm = nullptr;
  SBuf strong, weak, woff, ft[2], send, pend, cnt, out, qinfo;
  std::vector<std::vector<uint32_t>> h_weak;  // per local shard
  std::vector<std::vector<uint64_t>> h_woff;  // per local shard, absolute offsets, size nrounds+1
  bool weak_dirty = false;
  float last_ms = 0;
  uint64_t last_rounds = 0, last_xbytes = 0;
  std::string err;
  int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    err = buf;
    return code;
  }
};

#define SHCHK(c, x)                                                                                  \
  do {                                                                                               \
    hipError_t e_ = (x);                                                                             \
    if (e_ != hipSuccess) return (c)->fail(DR_E_HIP, "%s: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
  } while (0)

namespace {

int sh_set_device(dr_shard *c) {
  hipError_t e = hipSetDevice(c->dev);
  if (e != hipSuccess) return c->fail(DR_E_HIP, "hipSetDevice(%d): %s", c->dev, hipGetErrorString(e));
  return DR_OK;
}

// upload the weak edges appended since the last query (kept on the host until then)
int sync_weak(dr_shard *c) {
  if (!c->weak_dirty) return DR_OK;
  size_t total = 0;
  for (auto &v : c->h_weak) total += v.size();
  SHCHK(c, c->weak.ensure(std::max<size_t>(total, 1) * 4));
  SHCHK(c, c->woff.ensure((size_t)c->nlocal * (c->max_rounds + 1) * 8));
  std::vector<uint64_t> offs((size_t)c->nlocal * (c->max_rounds + 1), 0);
  size_t base = 0;
  for (int l = 0; l < c->nlocal; l++) {
    const auto &w = c->h_weak[l];
    if (!w.empty())
      SHCHK(c, hipMemcpyAsync(c->weak.as<uint32_t>() + base, w.data(), w.size() * 4, hipMemcpyHostToDevice, c->stream));
    uint64_t *o = &offs[(size_t)l * (c->max_rounds + 1)];
    for (int r = 0; r <= c->max_rounds; r++)
      o[r] = base + c->h_woff[l][std::min<size_t>(r, c->h_woff[l].size() - 1)];
    base += w.size();
  }
  SHCHK(c, hipMemcpyAsync(c->woff.p, offs.data(), offs.size() * 8, hipMemcpyHostToDevice, c->stream));
  SHCHK(c, hipStreamSynchronize(c->stream));
  c->weak_dirty = false;
  return DR_OK;
}

// one batch of <= 64 reach-set queries; rows land in host `out` at obase[i]
int sweep_batch(dr_shard *c, const std::vector<QInfo> &qs, const std::vector<size_t> &hbase, int strong_only,
                uint64_t *out) {
  const int nq = (int)qs.size();
  int T = 0, Bm = 1 << 30;
  int64_t words = 0;
  std::vector<QInfo> dq(qs);
  for (int i = 0; i < nq; i++) {
    T = std::max(T, qs[i].top);
    Bm = std::min(Bm, qs[i].bottom);
    dq[i].obase = words;
    words += (int64_t)(qs[i].top - qs[i].bottom + 1) * c->W;
  }
  const int NT = c->G * c->C;
  SHCHK(c, c->out.ensure(std::max<int64_t>(words, 1) * 8));
  SHCHK(c, c->qinfo.ensure(SH_BATCH * sizeof(QInfo)));
  SHCHK(c, hipMemcpyAsync(c->qinfo.p, dq.data(), nq * sizeof(QInfo), hipMemcpyHostToDevice, c->stream));
  SHCHK(c, hipMemsetAsync(c->pend.p, 0, (size_t)c->nlocal * c->depth * c->C * 8, c->stream));
  SHCHK(c, hipMemsetAsync(c->cnt.p, 0, (size_t)c->nlocal * 4, c->stream));
  std::vector<u64> ft0(NT, 0);
  for (int i = 0; i < nq; i++)
    if (qs[i].top == T && qs[i].src0 >= 0) ft0[qs[i].src0] |= 1ULL << i;
  SHCHK(c, hipMemcpyAsync(c->ft[T & 1].p, ft0.data(), (size_t)NT * 8, hipMemcpyHostToDevice, c->stream));

  ShardArgs a{};
  a.strong = c->strong.as<u64>();
  a.weak = c->weak.as<uint32_t>();
  a.woff = c->woff.as<uint64_t>();
  a.pend = c->pend.as<u64>();
  a.cnt = c->cnt.as<unsigned>();
  a.out = c->out.as<u64>();
  a.q = c->qinfo.as<QInfo>();
  a.n = c->n;
  a.W = c->W;
  a.WSs = c->WSs;
  a.C = c->C;
  a.depth = c->depth;
  a.shard0 = c->shard0;
  a.local = c->local ? 1 : 0;
  a.max_rounds = c->max_rounds;
  a.nq = nq;
  a.strong_only = strong_only;
  a.strong_shard_stride = (int64_t)c->max_rounds * c->n * c->WSs;
  const int item_waves = (c->n + 63) / 64 * c->WSs;  // (source chunk, target word) items
  const size_t weak_waves = strong_only ? 0 : (c->max_weak_round + 511) / 512;
  const int gx = (int)std::max<size_t>((item_waves + 3) / 4, std::min<size_t>(128, (weak_waves + 3) / 4));
  const dim3 grid(gx, c->nlocal), block(SH_NT);
  for (int r = T; r >= Bm; r--) {
    u64 expm = 0, outm = 0, injm = 0;
    for (int i = 0; i < nq; i++) {
      if (qs[i].bottom < r && r <= qs[i].top) expm |= 1ULL << i;
      if (qs[i].bottom <= r && r <= qs[i].top) outm |= 1ULL << i;
      if (qs[i].top == r - 1) injm |= 1ULL << i;
    }
    const int produce = r - 1 >= Bm;
    a.ft = c->ft[r & 1].as<u64>();
    a.ftn = c->local ? c->ft[(r - 1) & 1].as<u64>() : c->send.as<u64>();
    hipLaunchKernelGGL(k_shard_round, grid, block, 0, c->stream, a, r, expm, outm, injm, produce);
    SHCHK(c, hipGetLastError());
    if (produce && !c->local) {
      ncclResult_t nr = ncclAllGather(c->send.p, c->ft[(r - 1) & 1].p, (size_t)c->C, ncclUint64, c->comm, c->stream);
      if (nr != ncclSuccess) return c->fail(DR_E_RCCL, "ncclAllGather: %s", ncclGetErrorString(nr));
      c->last_xbytes += (uint64_t)c->C * 8;
    }
    c->last_rounds++;
  }
  std::vector<u64> tmp(words);
  SHCHK(c, hipMemcpyAsync(tmp.data(), c->out.p, words * 8, hipMemcpyDeviceToHost, c->stream));
  SHCHK(c, hipStreamSynchronize(c->stream));
  for (int i = 0; i < nq; i++)
    std::memcpy(out + hbase[i], &tmp[dq[i].obase], (size_t)(qs[i].top - qs[i].bottom + 1) * c->W * 8);
  return DR_OK;
}

// all queries, in batches of 64, timed with HIP events
int run_queries(dr_shard *c, const std::vector<QInfo> &qs, const std::vector<size_t> &hbase, int strong_only,
                uint64_t *out) {
  if (int rc = sync_weak(c)) return rc;
  c->last_rounds = 0;
  c->last_xbytes = 0;
  SHCHK(c, hipEventRecord(c->ev0, c->stream));
  for (size_t i0 = 0; i0 < qs.size(); i0 += SH_BATCH) {
    const size_t i1 = std::min(qs.size(), i0 + SH_BATCH);
    std::vector<QInfo> part(qs.begin() + i0, qs.begin() + i1);
    std::vector<size_t> hb(hbase.begin() + i0, hbase.begin() + i1);
    if (int rc = sweep_batch(c, part, hb, strong_only, out)) return rc;
  }
  SHCHK(c, hipEventRecord(c->ev1, c->stream));
  SHCHK(c, hipEventSynchronize(c->ev1));
  SHCHK(c, hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1));
  return DR_OK;
}

}  // namespace

extern "C" int dr_shard_unique_id(uint8_t *id) {
  if (!id) return DR_E_INVAL;
  ncclUniqueId u;
  ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) {
    g_shard_err = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
    return DR_E_RCCL;
  }
  static_assert(sizeof(ncclUniqueId) == DR_SHARD_ID_BYTES, "RCCL unique id size");
  std::memcpy(id, &u, sizeof u);
  return DR_OK;
}

extern "C" int dr_shard_create(int n, int faulty, int max_rounds, int device, int nshards, int rank, const uint8_t *id,
                               dr_shard **out) {
  if (!out) return DR_E_INVAL;
  *out = nullptr;
  if (n < 1 || n > 2048 || faulty < 0 || max_rounds < 1 || max_rounds > (1 << 20) || device < 0 || nshards < 1 ||
      nshards > 64 || rank < 0 || rank >= nshards || (!id && rank != 0)) {
    g_shard_err = "dr_shard_create: n in [1,2048], faulty >= 0, max_rounds in [1,2^20], device >= 0, "
                  "nshards in [1,64], 0 <= rank < nshards (rank 0 in local mode)";
    return DR_E_INVAL;
  }
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || device >= ndev) {
    g_shard_err = std::string("dr_shard_create: no usable HIP device (") +
                  (e != hipSuccess ? hipGetErrorString(e) : "ordinal out of range") + "); there is no CPU fallback";
    return DR_E_HIP;
  }
  dr_shard *c = new dr_shard();
  c->n = n;
  c->f = faulty;
  c->W = (n + 63) / 64;
  c->G = nshards;
  c->WSs = (c->W + nshards - 1) / nshards;
  c->C = c->WSs * 64;
  c->local = id == nullptr;
  c->shard0 = c->local ? 0 : rank;
  c->nlocal = c->local ? nshards : 1;
  c->max_rounds = max_rounds;
  c->dev = device;
  c->h_weak.resize(c->nlocal);
  c->h_woff.assign(c->nlocal, std::vector<uint64_t>(1, 0));
  if (sh_set_device(c) != DR_OK || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
    g_shard_err = "dr_shard_create: stream/event creation failed";
    dr_shard_destroy(c);
    return DR_E_HIP;
  }
  const size_t NT = (size_t)c->G * c->C;
  if (c->strong.ensure((size_t)c->nlocal * max_rounds * n * c->WSs * 8) != hipSuccess ||
      c->ft[0].ensure(NT * 8) != hipSuccess || c->ft[1].ensure(NT * 8) != hipSuccess ||
      c->send.ensure((size_t)c->C * 8) != hipSuccess || c->cnt.ensure(c->nlocal * 4) != hipSuccess) {
    g_shard_err = "dr_shard_create: device allocation failed";
    dr_shard_destroy(c);
    return DR_E_HIP;
  }
  if (!c->local) {
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    ncclResult_t r = ncclCommInitRank(&c->comm, nshards, u, rank);
    if (r != ncclSuccess) {
      g_shard_err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
      c->comm = nullptr;
      dr_shard_destroy(c);
      return DR_E_RCCL;
    }
  }
  *out = c;
  return DR_OK;
}

extern "C" void dr_shard_destroy(dr_shard *c) {
  if (!c) return;
  (void)hipSetDevice(c->dev);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  for (SBuf *b : {&c->strong, &c->weak, &c->woff, &c->ft[0], &c->ft[1], &c->send, &c->pend, &c->cnt, &c->out, &c->qinfo})
    b->release();
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

extern "C" const char *dr_shard_last_error(const dr_shard *c) { return c ? c->err.c_str() : g_shard_err.c_str(); }
extern "C" int dr_shard_num_rounds(const dr_shard *c) { return c ? c->nrounds : -1; }

extern "C" int dr_shard_info(const dr_shard *c, int *nshards, int *shard0, int *nlocal, int *col0, int *col1) {
  if (!c) return DR_E_INVAL;
  if (nshards) *nshards = c->G;
  if (shard0) *shard0 = c->shard0;
  if (nlocal) *nlocal = c->nlocal;
  if (col0) *col0 = std::min(c->n, c->shard0 * c->C) + 1;
  if (col1) *col1 = std::min(c->n, (c->shard0 + c->nlocal) * c->C) + 1;
  return DR_OK;
}

extern "C" int dr_shard_append_rounds_packed(dr_shard *c, int r0, int k, const uint32_t *slot_off,
                                             const uint16_t *slot_src, const uint64_t *strong,
                                             const uint32_t *weak_off, const uint32_t *weak_tgt) {
  if (!c) return DR_E_INVAL;
  if (int rc = sh_set_device(c)) return rc;
  if (r0 != c->nrounds) return c->fail(DR_E_STATE, "append at round %d but %d rounds mirrored", r0, c->nrounds);
  if (k < 0 || r0 + k > c->max_rounds) return c->fail(DR_E_INVAL, "append of %d rounds exceeds max_rounds %d", k, c->max_rounds);
  if (k == 0) return DR_OK;
  if (!slot_off || !slot_src || !strong || !weak_off) return c->fail(DR_E_INVAL, "null array");
  const int n = c->n, W = c->W, WSs = c->WSs, C = c->C;
  const u64 lastmask = (n % 64) ? ((1ULL << (n % 64)) - 1ULL) : ~0ULL;
  std::vector<u64> pres(W);
  std::vector<u64> rows((size_t)c->nlocal * k * n * WSs, 0);
  std::vector<std::vector<uint32_t>> wnew(c->nlocal);
  std::vector<std::vector<uint64_t>> wro(c->nlocal, std::vector<uint64_t>(k + 1, 0));
  int dmax = c->dmax;
  size_t maxw = c->max_weak_round;
  for (int i = 0; i < k; i++) {
    const int r = r0 + i;
    std::fill(pres.begin(), pres.end(), 0ULL);
    for (uint32_t sl = slot_off[i]; sl < slot_off[i + 1]; sl++) {
      const int s = slot_src[sl];
      if (s > n) return c->fail(DR_E_CONTRACT, "round %d slot %u: source %d > n=%d", r, sl - slot_off[i], s, n);
      if (s == 0) continue;
      const u64 bit = 1ULL << ((s - 1) & 63);
      if ((pres[(s - 1) >> 6] & bit) && r >= 1) return c->fail(DR_E_CONTRACT, "round %d: duplicate vertex id (%d,%d)", r, r, s);
      pres[(s - 1) >> 6] |= bit;
    }
    for (int l = 0; l < c->nlocal; l++) wro[l][i] = wnew[l].size();
    for (int s0 = 0; s0 < n; s0++) {
      const bool here = (pres[s0 >> 6] >> (s0 & 63)) & 1ULL;
      const uint64_t *row = strong + ((size_t)i * n + s0) * W;
      bool nz = false;
      for (int w = 0; w < W; w++) nz |= row[w] != 0;
      if (nz && !here) return c->fail(DR_E_CONTRACT, "round %d: strong edges on absent vertex (%d,%d)", r, r, s0 + 1);
      if (nz && r == 0) return c->fail(DR_E_CONTRACT, "round 0 vertex (0,%d) has strong edges", s0 + 1);
      if (row[W - 1] & ~lastmask) return c->fail(DR_E_CONTRACT, "round %d vertex (%d,%d): strong target source > n", r, r, s0 + 1);
      for (int l = 0; l < c->nlocal; l++) {
        const int g = c->shard0 + l;
        u64 *dst = &rows[(((size_t)l * k + i) * n + s0) * WSs];
        for (int w = 0; w < WSs; w++) {
          const int gw = g * WSs + w;
          dst[w] = gw < W ? row[gw] : 0ULL;
        }
      }
      const uint32_t ea = weak_off[(size_t)i * n + s0], eb = weak_off[(size_t)i * n + s0 + 1];
      if (eb < ea) return c->fail(DR_E_INVAL, "weak_off not monotone at round %d", r);
      if (eb > ea && !here) return c->fail(DR_E_CONTRACT, "round %d: weak edges on absent vertex (%d,%d)", r, r, s0 + 1);
      for (uint32_t e = ea; e < eb; e++) {
        const uint32_t t = weak_tgt[e];
        const int tr = (int)(t >> 11), ts = (int)(t & 2047u);
        if (ts >= n) return c->fail(DR_E_CONTRACT, "weak edge (%d,%d)->(%d,%d): source > n", r, s0 + 1, tr, ts + 1);
        if (tr > r - 2) return c->fail(DR_E_CONTRACT, "weak edge (%d,%d)->(%d,%d) must target a round < r-1", r, s0 + 1, tr, ts + 1);
        const int delta = r - tr;
        if (delta > 1023) return c->fail(DR_E_CONTRACT, "weak edge (%d,%d)->(%d,%d): delta %d > 1023 (sharded path)", r, s0 + 1, tr, ts + 1, delta);
        dmax = std::max(dmax, delta);
        const int l = ts / C - c->shard0;
        if (l < 0 || l >= c->nlocal) continue;  // another shard's column
        wnew[l].push_back(((uint32_t)delta << 22) | ((uint32_t)s0 << 11) | (uint32_t)(ts % C));
      }
    }
    for (int l = 0; l < c->nlocal; l++) {
      auto &w = wnew[l];
      // (delta, target) order inside the round: the kernel's wave-uniform OR path
      std::sort(w.begin() + wro[l][i], w.end(), [](uint32_t x, uint32_t y) {
        const uint32_t kx = ((x >> 22) << 11) | (x & 2047u), ky = ((y >> 22) << 11) | (y & 2047u);
        return kx < ky;
      });
      maxw = std::max<size_t>(maxw, w.size() - wro[l][i]);
    }
  }
  for (int l = 0; l < c->nlocal; l++) {
    wro[l][k] = wnew[l].size();
    const size_t dst = ((size_t)l * c->max_rounds + r0) * n * WSs;
    SHCHK(c, hipMemcpyAsync(c->strong.as<u64>() + dst, &rows[(size_t)l * k * n * WSs], (size_t)k * n * WSs * 8,
                            hipMemcpyHostToDevice, c->stream));
    const uint64_t base = c->h_weak[l].size();
    c->h_weak[l].insert(c->h_weak[l].end(), wnew[l].begin(), wnew[l].end());
    for (int i = 1; i <= k; i++) c->h_woff[l].push_back(base + wro[l][i]);
  }
  SHCHK(c, hipStreamSynchronize(c->stream));
  c->weak_dirty = true;
  c->dmax = dmax;
  int depth = 2;
  while (depth <= dmax) depth <<= 1;
  if (depth != c->depth || !c->pend.p) {
    SHCHK(c, c->pend.ensure((size_t)c->nlocal * depth * C * 8));
    c->depth = depth;
  }
  c->max_weak_round = maxw;
  c->nrounds += k;
  return DR_OK;
}

extern "C" int dr_shard_reach_sets(dr_shard *c, int q, const int32_t *from, const int32_t *bottom, int strong_only,
                                   uint64_t *out, size_t cap_words, size_t *out_words) {
  if (!c) return DR_E_INVAL;
  if (q < 0 || (q > 0 && (!from || !bottom))) return c->fail(DR_E_INVAL, "bad query arrays");
  if (int rc = sh_set_device(c)) return rc;
  size_t need = 0;
  std::vector<QInfo> qs(q);
  std::vector<size_t> hb(q);
  for (int i = 0; i < q; i++) {
    const int fr = from[2 * i], fs = from[2 * i + 1], b = bottom[i];
    if (fr < 0 || fr >= c->nrounds || b < 0 || b > fr)
      return c->fail(DR_E_INVAL, "query %d: rounds [%d,%d] outside the DAG", i, b, fr);
    qs[i] = QInfo{fr, b, (fs >= 1 && fs <= c->n) ? fs - 1 : -1, 0, 0};
    hb[i] = need;
    need += (size_t)(fr - b + 1) * c->W;
  }
  if (out_words) *out_words = need;
  if (need > cap_words || (!out && need)) return c->fail(DR_E_CAPACITY, "reach sets need %zu words", need);
  if (q == 0) return DR_OK;
  return run_queries(c, qs, hb, strong_only, out);
}

extern "C" int dr_shard_path_batch(dr_shard *c, int q, const int32_t *from, const int32_t *to, int strong_only,
                                   uint8_t *out) {
  if (!c) return DR_E_INVAL;
  if (q < 0 || (q > 0 && (!from || !to || !out))) return c->fail(DR_E_INVAL, "bad query arrays");
  if (int rc = sh_set_device(c)) return rc;
  std::vector<QInfo> qs;
  std::vector<size_t> hb;
  std::vector<int> idx;
  size_t need = 0;
  for (int i = 0; i < q; i++) {
    const int fr = from[2 * i], fs = from[2 * i + 1], tr = to[2 * i], ts = to[2 * i + 1];
    if (fr == tr && fs == ts) { out[i] = 1; continue; }  // process.go:91-93
    if (fr < 0 || fr >= c->nrounds)
      return c->fail(DR_E_INVAL, "query %d: from round %d outside the DAG (Go: index out of range)", i, fr);
    out[i] = 0;
    if (tr < 0 || tr >= fr || ts < 1 || ts > c->n || fs < 1 || fs > c->n) continue;
    // only the row of round tr is needed: a one-round output window
    qs.push_back(QInfo{fr, tr, fs - 1, 0, 0});
    hb.push_back(need);
    need += (size_t)(fr - tr + 1) * c->W;
    idx.push_back(i);
  }
  if (qs.empty()) return DR_OK;
  std::vector<uint64_t> sets(need);
  if (int rc = run_queries(c, qs, hb, strong_only, sets.data())) return rc;
  for (size_t k = 0; k < idx.size(); k++) {
    const int i = idx[k], ts = to[2 * i + 1] - 1;
    out[i] = (sets[hb[k] + (ts >> 6)] >> (ts & 63)) & 1ULL;  // round tr is the first row
  }
  return DR_OK;
}

extern "C" int dr_shard_stats(const dr_shard *c, float *ms, uint64_t *rounds, uint64_t *exchange_bytes) {
  if (!c) return DR_E_INVAL;
  if (ms) *ms = c->last_ms;
  if (rounds) *rounds = c->last_rounds;
  if (exchange_bytes) *exchange_bytes = c->last_xbytes;
  return DR_OK;
}
