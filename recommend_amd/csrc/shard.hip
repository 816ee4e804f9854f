// Row-sharded embedding tables across the ranks of one node: row id lives on rank
// id % world at local row id / world (the modulo spreads Zipf-hot ids over all GPUs).  The lookup is
//   route (bucket the ids by owner, stable) -> all-to-all ids -> gather local rows -> all-to-all rows
//   back -> unpermute,
// and the update sends the gradient rows the same way to their owners, which apply the sparse
// Adagrad on their shard.  The all-to-alls are RCCL (torch.distributed); these kernels are the
// on-device halves.  All are HBM-bound row moves (16-B accesses), deterministic.
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

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
  OT_REQUIRE(ids && perm && send_local && counts, "ot_shard_route: null operand");
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
