/*
 * build_walk.hip — the walk stream's hierarchy built on the device.
 *
 * scene.cpp walk_regroup re-groups the inner boxes of a sphere scene over the reference's leaf
 * sequence (bvh_node.rs:27-63 fixes the leaves and their order): top down, each
 * range of leaves is cut where SA(left) n_left + SA(right) n_right is least, ties going to the cut
 * nearest the middle (then the smaller cut).  This file makes the same cuts on the GPU, one launch per
 * level of the tree:
 *   - a workgroup per range of >= 2 leaves: a reverse block scan of the leaf boxes gives every suffix
 *     box, a forward scan every prefix box and with it the cost of every cut (in f64, the host's
 *     operations in the host's order: the costs are bit-identical); a block argmin under the total
 *     order (cost, distance to the middle, cut) picks the host's cut;
 *   - the range's node (pre-order index known from the leaf counts: left child = node + 1, right
 *     child = node + 2 n_left) is written, the two sub-ranges are appended to the next level's list;
 *   - a range of one leaf writes its leaf node.
 * The host then places and writes the records (walk_place_and_write, O(n)).  The result is the host
 * build's hierarchy node for node (tests/test_gpu_parity.py checks the walk streams byte for byte).
 */
#include <hip/hip_runtime.h>

#include <chrono>
#include <vector>

#include "kernel_common.h"

using namespace hrt;
using namespace hrt::host;

namespace {

struct DBox {
  float mn[3], mx[3];
};

struct DRange {
  uint32_t lo, hi, node, depth;
};

struct DNode {
  float mn[3], mx[3];
  int32_t leaf;
  uint32_t end, depth;
};

constexpr int BT = 256; /* threads per workgroup */

__device__ __forceinline__ DBox box_join(const DBox& a, const DBox& b) {
  DBox u;
  for (int k = 0; k < 3; k++) {
    u.mn[k] = fminf(a.mn[k], b.mn[k]);
    u.mx[k] = fmaxf(a.mx[k], b.mx[k]);
  }
  return u;
}

/* scene.cpp half_area: the same f64 operations in the same order */
__device__ __forceinline__ double half_area_d(const DBox& b) {
  const double x = (double)b.mx[0] - b.mn[0], y = (double)b.mx[1] - b.mn[1], z = (double)b.mx[2] - b.mn[2];
  return x * y + y * z + z * x;
}

/* inclusive block scan of boxes (Hillis-Steele over BT threads); reverse = suffix direction */
__device__ DBox block_scan(DBox v, DBox* sh, bool reverse) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int d = 1; d < BT; d <<= 1) {
    DBox o = v;
    const int src = reverse ? t + d : t - d;
    const bool has = reverse ? src < BT : src >= 0;
    if (has) o = box_join(v, sh[src]);
    __syncthreads();
    v = o;
    sh[t] = v;
    __syncthreads();
  }
  return v;
}

/* (cost, distance to the middle, cut): the order scene.cpp's sequential loop selects by */
__device__ __forceinline__ bool better(double c, uint32_t d, uint32_t k, double bc, uint32_t bd, uint32_t bk) {
  if (c != bc) return c < bc;
  if (d != bd) return d < bd;
  return k < bk;
}

__global__ __launch_bounds__(BT) void split_level(const DBox* __restrict__ leaves, DBox* __restrict__ suf,
                                                  const DRange* __restrict__ ranges, uint32_t n_ranges,
                                                  DRange* __restrict__ next, uint32_t* __restrict__ n_next,
                                                  DNode* __restrict__ nodes) {
  __shared__ DBox sh[BT];
  __shared__ double sc[BT];
  __shared__ uint32_t sd[BT], sk[BT];
  __shared__ DBox carry;
  const uint32_t r = blockIdx.x;
  if (r >= n_ranges) return;
  const DRange R = ranges[r];
  const uint32_t n = R.hi - R.lo;
  const int t = threadIdx.x;
  if (n == 1) {
    if (t == 0) {
      DNode& o = nodes[R.node];
      for (int k = 0; k < 3; k++) {
        o.mn[k] = leaves[R.lo].mn[k];
        o.mx[k] = leaves[R.lo].mx[k];
      }
      o.leaf = (int32_t)R.lo;
      o.end = R.node + 1;
      o.depth = R.depth;
    }
    return;
  }
  /* suffix boxes suf[lo + k] = union of leaves [lo + k, hi), chunks from the end */
  for (uint32_t base = 0; base < n; base += BT) {
    const uint32_t hi_k = n - 1 - base; /* this chunk covers k in (hi_k - BT, hi_k] */
    const int64_t k = (int64_t)hi_k - (BT - 1) + t;
    DBox v = leaves[R.lo + (k >= 0 ? (uint32_t)k : 0u)];
    if (k < 0) v = leaves[R.lo + hi_k]; /* padding: any box of the chunk leaves min/max unchanged */
    v = block_scan(v, sh, true);
    if (base > 0) v = box_join(v, carry);
    __syncthreads();
    if (t == 0) carry = v; /* the suffix of the chunk's first element carries to the next chunk */
    if (k >= 0) suf[R.lo + (uint32_t)k] = v;
    __syncthreads();
  }
  /* prefix boxes and the cost of every cut k (left = [lo, lo + k], right = the rest) */
  const uint32_t mid = (n - 1) / 2;
  double best_c = 0.0;
  uint32_t best_d = 0xFFFFFFFFu, best_k = 0xFFFFFFFFu;
  DBox whole;
  for (uint32_t base = 0; base < n; base += BT) {
    const uint32_t k = base + t;
    DBox v = leaves[R.lo + (k < n ? k : n - 1)];
    v = block_scan(v, sh, false);
    if (base > 0) v = box_join(v, carry);
    __syncthreads();
    if (t == BT - 1) carry = v;
    if (k == n - 1) whole = v;
    if (k + 1 < n) {
      const double c = half_area_d(v) * (double)(k + 1) + half_area_d(suf[R.lo + k + 1]) * (double)(n - 1 - k);
      const uint32_t d = k > mid ? k - mid : mid - k;
      if (best_k == 0xFFFFFFFFu || better(c, d, k, best_c, best_d, best_k)) {
        best_c = c;
        best_d = d;
        best_k = k;
      }
    }
    __syncthreads();
  }
  /* block argmin */
  sc[t] = best_c;
  sd[t] = best_d;
  sk[t] = best_k;
  __syncthreads();
  for (int s = BT / 2; s > 0; s >>= 1) {
    if (t < s && sk[t + s] != 0xFFFFFFFFu &&
        (sk[t] == 0xFFFFFFFFu || better(sc[t + s], sd[t + s], sk[t + s], sc[t], sd[t], sk[t]))) {
      sc[t] = sc[t + s];
      sd[t] = sd[t + s];
      sk[t] = sk[t + s];
    }
    __syncthreads();
  }
  if (((n - 1) % BT) == (uint32_t)t) { /* the thread that held k = n - 1 holds the whole box */
    const uint32_t cut = sk[0];
    DNode& o = nodes[R.node];
    for (int k = 0; k < 3; k++) {
      o.mn[k] = whole.mn[k];
      o.mx[k] = whole.mx[k];
    }
    o.leaf = -1;
    o.end = R.node + 2 * n - 1;
    o.depth = R.depth;
    const uint32_t slot = atomicAdd(n_next, 2u);
    next[slot] = DRange{R.lo, R.lo + cut + 1, R.node + 1, R.depth + 1};
    next[slot + 1] = DRange{R.lo + cut + 1, R.hi, R.node + 2 * (cut + 1), R.depth + 1};
  }
}

}  // namespace

namespace hrt {

void device_walk_regroup(const std::vector<WalkLeaf>& leaves, std::vector<WNode>& T, int device) {
  const uint32_t n = (uint32_t)leaves.size();
  T.clear();
  if (n == 0) return;
  int prev = -1;
  hip_check(hipGetDevice(&prev), "hipGetDevice");
  if (device >= 0) hip_check(hipSetDevice(device), "hipSetDevice");
  std::vector<DBox> hb(n);
  for (uint32_t i = 0; i < n; i++) {
    const Aabb& b = leaves[i].box;
    hb[i] = DBox{{b.mn.x, b.mn.y, b.mn.z}, {b.mx.x, b.mx.y, b.mx.z}};
  }
  const uint32_t n_nodes = 2 * n - 1;
  DBox *d_leaves = nullptr, *d_suf = nullptr;
  DRange* d_r[2] = {nullptr, nullptr};
  DNode* d_nodes = nullptr;
  uint32_t* d_cnt = nullptr;
  auto cleanup = [&] {
    (void)hipFree(d_leaves);
    (void)hipFree(d_suf);
    (void)hipFree(d_r[0]);
    (void)hipFree(d_r[1]);
    (void)hipFree(d_nodes);
    (void)hipFree(d_cnt);
    if (prev >= 0) (void)hipSetDevice(prev);
  };
  try {
    hip_check(hipMalloc((void**)&d_leaves, n * sizeof(DBox)), "hipMalloc(build)");
    hip_check(hipMalloc((void**)&d_suf, n * sizeof(DBox)), "hipMalloc(build)");
    hip_check(hipMalloc((void**)&d_r[0], (size_t)n * sizeof(DRange)), "hipMalloc(build)");
    hip_check(hipMalloc((void**)&d_r[1], (size_t)n * sizeof(DRange)), "hipMalloc(build)");
    hip_check(hipMalloc((void**)&d_nodes, (size_t)n_nodes * sizeof(DNode)), "hipMalloc(build)");
    hip_check(hipMalloc((void**)&d_cnt, sizeof(uint32_t)), "hipMalloc(build)");
    hip_check(hipMemcpy(d_leaves, hb.data(), n * sizeof(DBox), hipMemcpyHostToDevice), "hipMemcpy(build)");
    const DRange root{0u, n, 0u, 0u};
    hip_check(hipMemcpy(d_r[0], &root, sizeof(DRange), hipMemcpyHostToDevice), "hipMemcpy(build)");
    uint32_t count = 1, cur = 0;
    /* every level halves no range to nothing: at most n levels, in practice ~2 log2 n */
    for (uint32_t level = 0; count > 0 && level <= n; level++) {
      hip_check(hipMemset(d_cnt, 0, sizeof(uint32_t)), "hipMemset(build)");
      hipLaunchKernelGGL(split_level, dim3(count), dim3(BT), 0, 0, d_leaves, d_suf, d_r[cur], count, d_r[cur ^ 1],
                         d_cnt, d_nodes);
      hip_check(hipGetLastError(), "split_level launch");
      hip_check(hipMemcpy(&count, d_cnt, sizeof(uint32_t), hipMemcpyDeviceToHost), "hipMemcpy(build)");
      cur ^= 1;
    }
    std::vector<DNode> hn(n_nodes);
    hip_check(hipMemcpy(hn.data(), d_nodes, (size_t)n_nodes * sizeof(DNode), hipMemcpyDeviceToHost), "hipMemcpy(build)");
    T.resize(n_nodes);
    for (uint32_t i = 0; i < n_nodes; i++) {
      WNode& w = T[i];
      w.box.mn = v3(hn[i].mn[0], hn[i].mn[1], hn[i].mn[2]);
      w.box.mx = v3(hn[i].mx[0], hn[i].mx[1], hn[i].mx[2]);
      w.leaf = hn[i].leaf;
      w.end = hn[i].end;
      w.depth = hn[i].depth;
    }
  } catch (...) {
    cleanup();
    throw;
  }
  cleanup();
}

}  // namespace hrt
