// Row-sharded embedding tables across the ranks of one node: row id lives on rank
// id % world at local row id / world (the modulo spreads Zipf-hot ids over all GPUs).  The lookup is
//   route (bucket the ids by owner, stable) -> all-to-all ids -> gather local rows -> all-to-all rows
//   back -> unpermute,
// and the update sends the gradient rows the same way to their owners, which apply the sparse
// Adagrad on their shard.  ot_shard_route_unique routes each distinct id once (Zipf batches repeat
// hot ids: a C2-shape batch has ~175k distinct of 516k), so the ids, rows and gradient rows that
// cross xGMI shrink by that factor; ot_segment_rows_sum pre-sums the repeats' gradients.  The
// all-to-alls are RCCL (torch.distributed); these kernels are the on-device halves.  All are HBM-bound row moves (16-B accesses), deterministic.
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "common.h"

namespace ot {

// owner key and local row of every id; invalid ids go to owner 0 with local row -1 (zero rows)
__global__ void shard_keys_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t num_rows, int world,
                                  uint32_t* owner, int32_t* pos) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t id = ids[i];
  owner[i] = (id >= 0 && id < num_rows) ? (uint32_t)(id % world) : 0u;
  pos[i] = (int32_t)i;
}

// after the stable sort by owner: send_local[j] = local row of the j-th routed id, counts[owner]++
__global__ void shard_route_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t num_rows, int world,
                                   const uint32_t* __restrict__ owner_sorted, const int32_t* __restrict__ perm,
                                   int64_t* send_local, int32_t* counts) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int64_t id = ids[perm[j]];
  send_local[j] = (id >= 0 && id < num_rows) ? id / world : -1;
  // run boundaries of the sorted owner keys give the counts without atomics
  const uint32_t o = owner_sorted[j];
  if (j == n - 1 || owner_sorted[j + 1] != o) {
    // j is the last of its run; the run starts after the previous run's last element
    int64_t lo = 0, hi = j;                       // first index with owner_sorted == o
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (owner_sorted[mid] < o) lo = mid + 1; else hi = mid;
    }
    counts[o] = (int32_t)(j - lo + 1);
  }
}

__global__ void zero_i32_kernel(int32_t* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0;
}

// out[i] = table[idx[i]] (zeros for idx < 0): one float4 per thread
__global__ void gather_rows_kernel(const float* __restrict__ table, int E, const int64_t* __restrict__ idx,
                                   int64_t n, float* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int c4 = E / 4;
  if (t >= n * c4) return;
  const int64_t i = t / c4;
  const int c = 4 * (int)(t % c4);
  const int64_t r = idx[i];
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (r >= 0) v = *reinterpret_cast<const f32x4*>(table + r * E + c);
  *reinterpret_cast<f32x4*>(out + i * E + c) = v;
}

// inverse = 0: dst[j] = src[perm[j]] (to owner order); inverse = 1: dst[perm[j]] = src[j] (back)
__global__ void permute_rows_kernel(const float* __restrict__ src, const int32_t* __restrict__ perm, int64_t n,
                                    int E, int inverse, float* dst) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int c4 = E / 4;
  if (t >= n * c4) return;
  const int64_t j = t / c4;
  const int c = 4 * (int)(t % c4);
  const int64_t p = perm[j];
  if (inverse)
    *reinterpret_cast<f32x4*>(dst + p * E + c) = *reinterpret_cast<const f32x4*>(src + j * E + c);
  else
    *reinterpret_cast<f32x4*>(dst + j * E + c) = *reinterpret_cast<const f32x4*>(src + p * E + c);
}

// counter-based U(lo, hi) init of a shard: value of (global row id, column) independent of the
// sharding, so every world size builds the same logical table
__global__ void hash_uniform_rows_kernel(float* out, int64_t local_rows, int E, int rank, int world,
                                         uint32_t seed, float lo, float hi) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= local_rows * E) return;
  const int64_t r = t / E;
  const int c = (int)(t % E);
  const uint64_t gid = (uint64_t)(r * world + rank);
  const uint32_t h1 = fmix32((uint32_t)(gid * (uint64_t)E + c) * 0x9E3779B1u + seed);
  const uint32_t h2 = fmix32(h1 ^ (uint32_t)(gid >> 32) ^ 0x85EBCA77u);
  const float u = (float)(h2 >> 8) * (1.f / 16777216.f);
  out[t] = lo + (hi - lo) * u;
}

struct RouteWs {
  uint32_t *owner_in, *owner_out;
  int32_t *pos_in;
  void* tmp;
  size_t tmp_bytes, total;
};

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// ---- de-duplicating route (ot_shard_route_unique) -----------------------------------------
// Sort key of an id: owner in bits 40.., local row + 1 in bits 0..39 (invalid ids: owner 0, 0), so
// one radix sort orders the ids by owner and brings equal ids together; the stable sort keeps the
// original positions ascending inside every run (fixed summation order for ot_segment_rows_sum).
constexpr int UKEY_LOCAL_BITS = 40;

__global__ void ukeys_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t num_rows, int world, uint64_t* key,
                             int32_t* pos) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t id = ids[i];
  const bool ok = id >= 0 && id < num_rows;
  key[i] = ok ? ((uint64_t)(id % world) << UKEY_LOCAL_BITS) | (uint64_t)(id / world + 1) : 0ull;
  pos[i] = (int32_t)i;
}

// head[j] = 1 where sorted key j starts a run of equal ids
__global__ void uheads_kernel(const uint64_t* __restrict__ ks, int64_t n, int32_t* head) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  head[j] = (j == 0 || ks[j] != ks[j - 1]) ? 1 : 0;
}

// uidx[j] = inclusive count of heads (unique index + 1).  Writes inv (token -> unique), the unique
// ids' local rows, the run starts (run_start[U] = n) and per-owner unique counts (run boundaries of
// the sorted owner field, no atomics).
__global__ void ufinish_kernel(const uint64_t* __restrict__ ks, const int32_t* __restrict__ order,
                               const int32_t* __restrict__ uidx, int64_t n, int64_t* inv, int64_t* uniq_local,
                               int32_t* run_start, int32_t* counts) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint64_t k = ks[j];
  const int32_t u = uidx[j] - 1;
  inv[order[j]] = u;
  if (j == 0 || k != ks[j - 1]) {
    uniq_local[u] = (int64_t)(k & ((1ull << UKEY_LOCAL_BITS) - 1)) - 1;
    run_start[u] = (int32_t)j;
  }
  if (j == n - 1) run_start[u + 1] = (int32_t)n;
  const uint64_t o = k >> UKEY_LOCAL_BITS;
  if (j == n - 1 || (ks[j + 1] >> UKEY_LOCAL_BITS) != o) {
    int64_t lo = 0, hi = j;                       // first sorted index of owner o
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if ((ks[mid] >> UKEY_LOCAL_BITS) < o) lo = mid + 1; else hi = mid;
    }
    counts[o] = uidx[j] - (lo > 0 ? uidx[lo - 1] : 0);
  }
}

// out[u] = sum of src[order[j]] over j in [run_start[u], run_start[u + 1]), ascending j: one float4
// column of one unique row per thread
__global__ void segment_rows_sum_kernel(const float* __restrict__ src, const int32_t* __restrict__ order,
                                        const int32_t* __restrict__ run_start, int64_t U, int E, float* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int c4 = E / 4;
  if (t >= U * c4) return;
  const int64_t u = t / c4;
  const int c = 4 * (int)(t % c4);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int32_t j = run_start[u]; j < run_start[u + 1]; ++j)
    acc += *reinterpret_cast<const f32x4*>(src + (int64_t)order[j] * E + c);
  *reinterpret_cast<f32x4*>(out + u * E + c) = acc;
}

// Balanced form (ot_segment_rows_sum_ex): Zipf batches repeat hot ids tens of thousands of times, and
// one thread per (distinct id, float4 column) then walks a hot id's whole run alone (C4: 12.8 ms per
// step in one launch).  Each run is cut into pieces of at most SEG_PIECE positions (piece offsets =
// exclusive scan of the per-run piece counts); one thread per (piece, float4 column) sums its piece in
// ascending position order, and a run of several pieces adds its pieces' partials in piece order
// (fixed: deterministic).  A run of one piece is written straight to out.
constexpr int SEG_PIECE = 64;

__global__ void seg_piece_count_kernel(const int32_t* __restrict__ run_start, int64_t U, int32_t* cnt) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= U) return;
  cnt[u] = (run_start[u + 1] - run_start[u] + SEG_PIECE - 1) / SEG_PIECE;
}

__global__ void seg_piece_sum_kernel(const float* __restrict__ src, const int32_t* __restrict__ order,
                                     const int32_t* __restrict__ run_start, const int32_t* __restrict__ cnt,
                                     const int32_t* __restrict__ poff, int64_t U, int64_t pmax, int E,
                                     float* partial, float* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int c4 = E / 4;
  if (t >= pmax * c4) return;
  const int64_t p = t / c4;
  const int c = 4 * (int)(t % c4);
  if (p >= (int64_t)poff[U - 1] + cnt[U - 1]) return;         // past the last piece
  int64_t lo = 0, hi = U - 1;                                  // run u: poff[u] <= p < poff[u + 1]
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (poff[mid] <= p) lo = mid; else hi = mid - 1;
  }
  const int64_t u = lo;
  const int32_t q = (int32_t)(p - poff[u]);
  const int32_t j0 = run_start[u] + q * SEG_PIECE;
  const int32_t j1 = min(run_start[u + 1], j0 + SEG_PIECE);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int32_t j = j0; j < j1; ++j) acc += *reinterpret_cast<const f32x4*>(src + (int64_t)order[j] * E + c);
  float* dst = cnt[u] == 1 ? out + u * E : partial + p * E;
  *reinterpret_cast<f32x4*>(dst + c) = acc;
}

__global__ void seg_piece_final_kernel(const float* __restrict__ partial, const int32_t* __restrict__ cnt,
                                       const int32_t* __restrict__ poff, int64_t U, int E, float* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int c4 = E / 4;
  if (t >= U * c4) return;
  const int64_t u = t / c4;
  const int np = cnt[u];
  if (np <= 1) return;
  const int c = 4 * (int)(t % c4);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int q = 0; q < np; ++q) acc += *reinterpret_cast<const f32x4*>(partial + ((int64_t)poff[u] + q) * E + c);
  *reinterpret_cast<f32x4*>(out + u * E + c) = acc;
}

struct SegWs {
  int32_t *cnt, *poff;
  float* partial;
  void* scan_tmp;
  size_t scan_bytes, total;
};

SegWs carve_seg(void* base, int64_t U, int64_t n, int E) {
  SegWs w{};
  (void)rocprim::exclusive_scan(nullptr, w.scan_bytes, (int32_t*)nullptr, (int32_t*)nullptr, 0, (size_t)U,
                                rocprim::plus<int32_t>());
  char* p = (char*)base;
  size_t off = 0;
  auto take = [&](size_t bytes) { char* r = p ? p + off : nullptr; off += al256(bytes); return (void*)r; };
  const int64_t pmax = U + n / SEG_PIECE + 1;
  w.cnt = (int32_t*)take(U * 4);
  w.poff = (int32_t*)take(U * 4);
  w.partial = (float*)take(pmax * E * 4);
  w.scan_tmp = take(w.scan_bytes);
  w.total = off;
  return w;
}

struct URouteWs {
  uint64_t *key_in, *key_out;
  int32_t *pos_in, *head, *uidx;
  void *sort_tmp, *scan_tmp;
  size_t sort_bytes, scan_bytes, total;
};

URouteWs carve_uroute(void* base, int64_t n) {
  URouteWs w{};
  (void)rocprim::radix_sort_pairs(nullptr, w.sort_bytes, (uint64_t*)nullptr, (uint64_t*)nullptr, (int32_t*)nullptr,
                                  (int32_t*)nullptr, (size_t)n, 0, 64);
  (void)rocprim::inclusive_scan(nullptr, w.scan_bytes, (int32_t*)nullptr, (int32_t*)nullptr, (size_t)n,
                                rocprim::plus<int32_t>());
  char* p = (char*)base;
  size_t off = 0;
  auto take = [&](size_t bytes) { char* r = p ? p + off : nullptr; off += al256(bytes); return (void*)r; };
  w.key_in = (uint64_t*)take(n * 8);
  w.key_out = (uint64_t*)take(n * 8);
  w.pos_in = (int32_t*)take(n * 4);
  w.head = (int32_t*)take(n * 4);
  w.uidx = (int32_t*)take(n * 4);
  w.sort_tmp = take(w.sort_bytes);
  w.scan_tmp = take(w.scan_bytes);
  w.total = off;
  return w;
}

RouteWs carve_route(void* base, int64_t n) {
  RouteWs w{};
  size_t sort_bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, sort_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr, (int32_t*)nullptr,
                                  (int32_t*)nullptr, (size_t)n, 0, 32);
  w.tmp_bytes = sort_bytes;
  char* p = (char*)base;
  size_t off = 0;
  auto take = [&](size_t bytes) { char* r = p ? p + off : nullptr; off += al256(bytes); return (void*)r; };
  w.owner_in = (uint32_t*)take(n * 4);
  w.owner_out = (uint32_t*)take(n * 4);
  w.pos_in = (int32_t*)take(n * 4);
  w.tmp = take(w.tmp_bytes);
  w.total = off;
  return w;
}

}  // namespace ot

using namespace ot;

extern "C" size_t ot_shard_route_workspace_size(int64_t n) { return n > 0 ? carve_route(nullptr, n).total : 256; }

extern "C" int ot_shard_route(const int64_t* ids, int64_t n, int64_t num_rows, int world, int32_t* perm,
                              int64_t* send_local, int32_t* counts, void* workspace, size_t ws_bytes, void* stream) {
  OT_REQUIRE((ids || n == 0) && perm && send_local && counts, "ot_shard_route: null operand");
  OT_REQUIRE(world >= 1 && world <= 1024, "ot_shard_route: world %d out of range", world);
  OT_REQUIRE(n >= 0 && n < 2147483647LL && num_rows > 0, "ot_shard_route: bad sizes");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(zero_i32_kernel, dim3(ceil_div(world, 256)), dim3(256), 0, s, counts, world);
  if (n == 0) return OT_OK;
  RouteWs w = carve_route(workspace, n);
  OT_REQUIRE(ws_bytes >= w.total, "ot_shard_route: workspace too small (%zu < %zu)", ws_bytes, w.total);
  const unsigned g = ceil_div(n, 256);
  hipLaunchKernelGGL(shard_keys_kernel, dim3(g), dim3(256), 0, s, ids, n, num_rows, world, w.owner_in, w.pos_in);
  OT_LAUNCH_CHECK("ot_shard_route(keys)");
  int end_bit = 1;
  while ((1 << end_bit) < world) ++end_bit;
  size_t tb = w.tmp_bytes;
  hipError_t e = rocprim::radix_sort_pairs(w.tmp, tb, w.owner_in, w.owner_out, w.pos_in, perm, (size_t)n, 0, end_bit,
                                           s);
  if (e != hipSuccess) return fail(OT_ERR_HIP, "ot_shard_route(sort): %s", hipGetErrorString(e));
  hipLaunchKernelGGL(shard_route_kernel, dim3(g), dim3(256), 0, s, ids, n, num_rows, world, w.owner_out, perm,
                     send_local, counts);
  OT_LAUNCH_CHECK("ot_shard_route(route)");
  return OT_OK;
}

extern "C" size_t ot_shard_route_unique_workspace_size(int64_t n) {
  return n > 0 ? carve_uroute(nullptr, n).total : 256;
}

extern "C" int ot_shard_route_unique(const int64_t* ids, int64_t n, int64_t num_rows, int world, int64_t* uniq_local,
                                     int64_t* inv, int32_t* order, int32_t* run_start, int32_t* counts,
                                     void* workspace, size_t ws_bytes, void* stream) {
  OT_REQUIRE((ids || n == 0) && uniq_local && inv && order && run_start && counts,
             "ot_shard_route_unique: null operand");
  OT_REQUIRE(world >= 1 && world <= 1024, "ot_shard_route_unique: world %d out of range", world);
  OT_REQUIRE(n >= 0 && n < 2147483647LL, "ot_shard_route_unique: bad n");
  OT_REQUIRE(num_rows > 0 && num_rows / world + 1 < (1LL << UKEY_LOCAL_BITS),
             "ot_shard_route_unique: num_rows out of range");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(zero_i32_kernel, dim3(ceil_div(world, 256)), dim3(256), 0, s, counts, world);
  if (n == 0) {
    hipLaunchKernelGGL(zero_i32_kernel, dim3(1), dim3(256), 0, s, run_start, 1);
    OT_LAUNCH_CHECK("ot_shard_route_unique(empty)");
    return OT_OK;
  }
  URouteWs w = carve_uroute(workspace, n);
  OT_REQUIRE(ws_bytes >= w.total, "ot_shard_route_unique: workspace too small (%zu < %zu)", ws_bytes, w.total);
  const unsigned g = ceil_div(n, 256);
  hipLaunchKernelGGL(ukeys_kernel, dim3(g), dim3(256), 0, s, ids, n, num_rows, world, w.key_in, w.pos_in);
  OT_LAUNCH_CHECK("ot_shard_route_unique(keys)");
  int end_bit = UKEY_LOCAL_BITS;
  while ((1 << (end_bit - UKEY_LOCAL_BITS)) < world) ++end_bit;
  size_t sb = w.sort_bytes;
  hipError_t e = rocprim::radix_sort_pairs(w.sort_tmp, sb, w.key_in, w.key_out, w.pos_in, order, (size_t)n, 0,
                                           end_bit, s);
  if (e != hipSuccess) return fail(OT_ERR_HIP, "ot_shard_route_unique(sort): %s", hipGetErrorString(e));
  hipLaunchKernelGGL(uheads_kernel, dim3(g), dim3(256), 0, s, w.key_out, n, w.head);
  OT_LAUNCH_CHECK("ot_shard_route_unique(heads)");
  size_t cb = w.scan_bytes;
  e = rocprim::inclusive_scan(w.scan_tmp, cb, w.head, w.uidx, (size_t)n, rocprim::plus<int32_t>(), s);
  if (e != hipSuccess) return fail(OT_ERR_HIP, "ot_shard_route_unique(scan): %s", hipGetErrorString(e));
  hipLaunchKernelGGL(ufinish_kernel, dim3(g), dim3(256), 0, s, w.key_out, order, w.uidx, n, inv, uniq_local,
                     run_start, counts);
  OT_LAUNCH_CHECK("ot_shard_route_unique(finish)");
  return OT_OK;
}

extern "C" int ot_segment_rows_sum(const float* src, const int32_t* order, const int32_t* run_start, int64_t U, int E,
                                   float* out, void* stream) {
  OT_REQUIRE(src && order && run_start && out && E > 0 && E % 4 == 0 && U >= 0, "ot_segment_rows_sum: bad args");
  if (U == 0) return OT_OK;
  hipLaunchKernelGGL(segment_rows_sum_kernel, dim3(ceil_div(U * (E / 4), 256)), dim3(256), 0, (hipStream_t)stream,
                     src, order, run_start, U, E, out);
  OT_LAUNCH_CHECK("ot_segment_rows_sum");
  return OT_OK;
}

extern "C" size_t ot_segment_rows_sum_workspace_size(int64_t U, int64_t n, int E) {
  return U > 0 && n >= U && E > 0 ? carve_seg(nullptr, U, n, E).total : 256;
}

extern "C" int ot_segment_rows_sum_ex(const float* src, const int32_t* order, const int32_t* run_start, int64_t U,
                                      int64_t n, int E, float* out, void* workspace, size_t ws_bytes, void* stream) {
  OT_REQUIRE(src && order && run_start && out && E > 0 && E % 4 == 0 && U >= 0 && n >= U && n < 2147483647LL,
             "ot_segment_rows_sum_ex: bad args");
  if (U == 0) return OT_OK;
  SegWs w = carve_seg(workspace, U, n, E);
  OT_REQUIRE(workspace && ws_bytes >= w.total, "ot_segment_rows_sum_ex: workspace too small (%zu < %zu)", ws_bytes,
             w.total);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(seg_piece_count_kernel, dim3(ceil_div(U, 256)), dim3(256), 0, s, run_start, U, w.cnt);
  OT_LAUNCH_CHECK("ot_segment_rows_sum_ex(count)");
  size_t sb = w.scan_bytes;
  hipError_t e = rocprim::exclusive_scan(w.scan_tmp, sb, w.cnt, w.poff, 0, (size_t)U, rocprim::plus<int32_t>(), s);
  if (e != hipSuccess) return fail(OT_ERR_HIP, "ot_segment_rows_sum_ex(scan): %s", hipGetErrorString(e));
  const int64_t pmax = U + n / SEG_PIECE + 1;
  hipLaunchKernelGGL(seg_piece_sum_kernel, dim3(ceil_div(pmax * (E / 4), 256)), dim3(256), 0, s, src, order, run_start,
                     w.cnt, w.poff, U, pmax, E, w.partial, out);
  OT_LAUNCH_CHECK("ot_segment_rows_sum_ex(pieces)");
  hipLaunchKernelGGL(seg_piece_final_kernel, dim3(ceil_div(U * (E / 4), 256)), dim3(256), 0, s, w.partial, w.cnt,
                     w.poff, U, E, out);
  OT_LAUNCH_CHECK("ot_segment_rows_sum_ex(final)");
  return OT_OK;
}

extern "C" int ot_gather_rows(const float* table, int E, const int64_t* idx, int64_t n, float* out, void* stream) {
  OT_REQUIRE(table && idx && out && E > 0 && E % 4 == 0, "ot_gather_rows: bad args");
  if (n <= 0) return OT_OK;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(ceil_div(n * (E / 4), 256)), dim3(256), 0, (hipStream_t)stream, table,
                     E, idx, n, out);
  OT_LAUNCH_CHECK("ot_gather_rows");
  return OT_OK;
}

extern "C" int ot_permute_rows(const float* src, const int32_t* perm, int64_t n, int E, int inverse, float* dst,
                               void* stream) {
  OT_REQUIRE(src && perm && dst && E > 0 && E % 4 == 0, "ot_permute_rows: bad args");
  if (n <= 0) return OT_OK;
  hipLaunchKernelGGL(permute_rows_kernel, dim3(ceil_div(n * (E / 4), 256)), dim3(256), 0, (hipStream_t)stream, src,
                     perm, n, E, inverse, dst);
  OT_LAUNCH_CHECK("ot_permute_rows");
  return OT_OK;
}

extern "C" int ot_hash_uniform_rows(float* out, int64_t local_rows, int E, int rank, int world, uint32_t seed,
                                    float lo, float hi, void* stream) {
  OT_REQUIRE(out && E > 0 && world >= 1 && rank >= 0 && rank < world, "ot_hash_uniform_rows: bad args");
  if (local_rows <= 0) return OT_OK;
  hipLaunchKernelGGL(hash_uniform_rows_kernel, dim3(ceil_div(local_rows * E, 256)), dim3(256), 0, (hipStream_t)stream,
                     out, local_rows, E, rank, world, seed, lo, hi);
  OT_LAUNCH_CHECK("ot_hash_uniform_rows");
  return OT_OK;
}
