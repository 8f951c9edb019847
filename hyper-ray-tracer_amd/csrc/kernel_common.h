/*
 * kernel_common.h — what the kernel translation units share: the work claim, LDS staging, sample
 * accumulation and counters of the persistent kernels (device), and the host helpers of the device
 * runtime.  render.hip holds the general kernels and the runtime; render_sphere.hip the sphere-scene
 * kernel, compiled on its own (Makefile: without the SLP vectorizer, which pairs its box-test
 * arithmetic into v_pk_* operations that measured slower).
 */
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "scene_internal.h"
#include "lane.h"

namespace hrt {

/* host side (render.hip) */
struct HipError {
  hrt_status code;
  std::string msg;
};
void hip_check(hipError_t e, const char* what);
/* persistent grid: as many workgroups as are co-resident on the device (cached per kernel/device) */
/* the persistent grid of a kernel (occupancy x CUs, cached); records the launch for hrt_last_launch
 * (`name`: the launcher's __PRETTY_FUNCTION__, whose template arguments name the instantiation) */
int resident_grid(const void* fn, int block, int device, size_t smem, bool lds, const char* name);
/* render_sphere.hip: launch render_basic_kernel<cull, count, lds> */
void launch_sphere(int cull, bool count, bool lds, bool heavy, bool packet, const lane::KParams& kp, int device,
                   hipStream_t stream, size_t smem);
/* render_general.hip: launch render_gwalk_kernel (wmem: lane.h WM_*, lref: reference stream in LDS,
 * trim: lane.h TRIM_* features compiled out) */
void launch_gwalk(bool count, int wmem, bool lref, int trim, bool one, bool packet, const lane::KParams& kp, int device,
                  hipStream_t stream, size_t smem);

namespace kern {
namespace G = hrt::gpu;
using namespace hrt::lane;

/* COUNT builds of the sphere-scene kernel: shader-clock cycles per wave phase (s_memtime stamps,
 * uniform per wave): [0] claim + sample start, [1] walk, [2] shading */
/* The walk kernels recompute the ray's derived fields (1/d, the inflated test's origin term, d.d, RN(1/d.d):
 * lane.h set_dir) for EVERY lane at the top of every pass, the same bits again for a lane in mid-walk: they
 * are then dead across the shading code, which otherwise keeps them in registers (or scratch) for the lanes
 * still walking.  The wave runs set_dir's instructions each pass for its new rays anyway.  0: only new rays
 * (A/B; profiles/r04g_ab.txt). */
#ifndef HRT_RAY_REDERIVE
#define HRT_RAY_REDERIVE 1 /* the general kernel (r04: Cornell-smoke +4.9%, Final neutral, bit-identical) */
#endif
#ifndef HRT_RAY_REDERIVE_SPHERE
#define HRT_RAY_REDERIVE_SPHERE 0 /* the sphere kernel (r04: C2 -3%, C3 -0.7%: its shading spills nothing) */
#endif

struct PhaseClock {
  unsigned long long cyc[3];
  unsigned long long last;
  unsigned long long leaf; /* inside cyc[1]: the batched leaf-test blocks (hrt_render_stats.leaf_cycles) */
};

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}

/* ------------------------------------------------------------------ the megakernel */
/* LDS: the node stream and primitive records are copied into LDS once per workgroup (they are
 * read ~60 times per ray by dependent loads; LDS latency is a fraction of an L2 hit). */
template <bool LDS, bool FAST>
constexpr int block_threads() { return LDS ? (FAST ? 1024 : 512) : 256; }

/* LDS staging of n Perlin tables at dst (an LDS address that is a multiple of PERLIN_LDS_ALIGN; layout.h Perlin).
 * HRT_PERLIN_XADDR (default): each permutation word v becomes v << 4, its ranvec entry's byte offset in the table
 * (< 4096), and the x permutation's also carries the table's own LDS address (a multiple of 4096), so the gradient
 * of a lattice corner is at LDS address px ^ py ^ pz (lane.h perlin_noise_t<true>): the three words XOR to the
 * address with no shift and add per corner. */
__device__ __forceinline__ const G::Perlin* stage_perlin(float4* dst, const G::Perlin* src, uint32_t n) {
  const float4* g = reinterpret_cast<const float4*>(src);
  constexpr uint32_t PER = (uint32_t)(sizeof(G::Perlin) / 16u), RV = 256u, PW = G::PERM_N / 4u; /* float4s */
  const uint32_t n4 = n * PER;
  const uint32_t at = (uint32_t)(size_t)(__attribute__((address_space(3))) float4*)dst;
  for (uint32_t k = threadIdx.x; k < n4; k += blockDim.x) {
    float4 v = g[k];
#if HRT_PERLIN_XADDR
    const uint32_t t = k / PER, w = k - t * PER;
    if (w >= RV && w < RV + 3u * PW) {
      const uint32_t base = w < RV + PW ? at + t * (uint32_t)sizeof(G::Perlin) : 0u;
      v = make_float4(__uint_as_float((__float_as_uint(v.x) << 4) | base), __uint_as_float((__float_as_uint(v.y) << 4) | base),
                      __uint_as_float((__float_as_uint(v.z) << 4) | base), __uint_as_float((__float_as_uint(v.w) << 4) | base));
    }
#endif
    dst[k] = v;
  }
  return reinterpret_cast<const G::Perlin*>(dst);
}

/* the LDS float4 at or after p whose address is a multiple of a (dynamic LDS) */
__device__ __forceinline__ float4* lds_align(float4* p, uint32_t a) {
  const uint32_t at = (uint32_t)(size_t)(__attribute__((address_space(3))) float4*)p;
  return p + (((at + a - 1u) & ~(a - 1u)) - at) / 16u;
}

/* Copy the node stream and primitive records into this workgroup's LDS.  BYTE_LINKS: store each skip
 * link as the LDS byte address of its target (base + skip x sizeof(Node)), for walks whose position is
 * that address (basic_box STRIDE 32). */
template <bool BYTE_LINKS = false>
__device__ __forceinline__ void stage_scene(const KParams& P, float4* lds, const G::Node*& nodes, const G::Prim*& prims,
                                            uint32_t base = 0u) {
  const uint32_t n4 = P.n_nodes * (uint32_t)(sizeof(G::Node) / 16);
  const uint32_t p4 = P.n_prims * (uint32_t)(sizeof(G::Prim) / 16);
  const float4* gn = reinterpret_cast<const float4*>(P.nodes);
  const float4* gp = reinterpret_cast<const float4*>(P.prims);
  for (uint32_t k = threadIdx.x; k < n4; k += blockDim.x) {
    float4 v = gn[k];
    if (BYTE_LINKS && (k & 1u) == 0u) v.w = __uint_as_float(base + __float_as_uint(v.w) * (uint32_t)sizeof(G::Node));
    lds[k] = v;
  }
  for (uint32_t k = threadIdx.x; k < p4; k += blockDim.x) lds[n4 + k] = gp[k];
  __syncthreads();
  nodes = reinterpret_cast<const G::Node*>(lds);
  prims = reinterpret_cast<const G::Prim*>(lds + n4);
}

/* A lane's current work item: one pixel and a chunk [sample, sample_end) of its samples.  slot: where
 * the chunk's result goes, P.out[slot] (one chunk) or P.partial[slot] = [chunk][n_out] (the host checks
 * n_chunks x n_out < 2^32); the chunk is first iff sample_end <= P.chunk (lane.h chunk_plan). */
struct Item {
  uint32_t pxy; /* px | py << 16 */
  uint32_t slot, sample, sample_end;
};

/* Work items claimed by a wave and not yet handed to a lane: [next, end) (wave-uniform). */
struct WaveBlock {
  uint32_t next, end;
};
constexpr uint32_t CLAIM_BLOCK = 64; /* items per atomicAdd on the work counter */

/* Idle lanes of the wave take work items from the wave's block (ballot + popcount); when it runs short
 * the wave claims the next CLAIM_BLOCK items with ONE atomicAdd.  Items are the head chunks' (lane.h
 * chunk_plan) ordered [tile][8x8 block][chunk][64 pixels], then the short tail chunks' chunk-major, so
 * the launch ends on short items; a block is one chunk of 64 neighbouring pixels.  A wave hands out its whole block before it claims another,
 * and its lanes retire only on an item past the end, so no item is left behind. */
/* RECOMPUTE (the general walk kernel): the work division's uniform divisors pass through an opaque copy at every
 * claim, so their reciprocals are computed where a claim needs them instead of being kept in vector registers
 * across the whole persistent loop (the general kernel at its 128-VGPR cap spilled them; claims are rare next to
 * node steps).  The lane's rank among the claiming lanes comes from v_mbcnt (no per-lane mask kept live). */
#ifndef HRT_CLAIM_MBCNT
#define HRT_CLAIM_MBCNT 1
#endif
template <bool RECOMPUTE = false>
__device__ __forceinline__ void claim_work(const KParams& P, uint32_t lane, bool& has_item, bool& exhausted,
                                           Item& it, WaveBlock& wb) {
  const bool want = !has_item && !exhausted;
  const unsigned long long want_mask = __ballot(want);
  if (!want_mask) return;
  const uint32_t cnt = (uint32_t)__popcll(want_mask);
#if HRT_CLAIM_MBCNT
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(want_mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)want_mask, 0u));
#else
  const uint32_t rank = (uint32_t)__popcll(want_mask & ((1ull << lane) - 1ull));
#endif
  const uint32_t avail = wb.end - wb.next;
  uint32_t w = wb.next + rank;
  if (cnt > avail) { /* the block's rest, then a new block (cnt <= 64 = CLAIM_BLOCK) */
    /* the frame's last items go one per lane again (P.claim_fine), so no wave sits on a block while
     * other waves idle at the end */
    const uint32_t size = wb.end >= P.claim_fine ? cnt - avail : CLAIM_BLOCK;
    const int leader = __ffsll((long long)want_mask) - 1;
    uint32_t base = 0;
#if HRT_CLAIM_MBCNT
    /* the leader is the wanting lane of rank 0 (no lane index kept live); its result read back by a readlane */
    if (want && rank == 0u) base = atomicAdd(P.counter, size);
    base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);
#else
    if ((int)lane == leader) base = atomicAdd(P.counter, size);
    base = __builtin_amdgcn_readfirstlane(__shfl(base, leader));
#endif
    if (rank >= avail) w = base + (rank - avail);
    wb.next = base + (cnt - avail);
    wb.end = base + size;
  } else {
    wb.next += cnt;
  }
  if (!want) return;
  if (w >= P.total_work) {
    exhausted = true;
    return;
  }
  /* head items [tile][8x8 block][head chunk][64 pixels] (a wave works through one block's chunks in a
   * row: its pixels' texels and partial sums stay in cache), then the tail items chunk-major
   * [tail chunk][tile][8x8 block][64 pixels]; px = the padded pixel, then its tile (tiles padded to one
   * stride: a division; else a binary search on pad_start) */
  uint32_t chunk_head = P.chunk_head, pad_px = P.pad_px, tile_stride = P.tile_stride;
  if constexpr (RECOMPUTE) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(chunk_head), "+s"(pad_px), "+s"(tile_stride));
#endif
  }
  uint32_t c, px;
  if (w < P.head_items) {
    const uint32_t g = w / (64u * chunk_head), rem = w - g * 64u * chunk_head;
    c = rem >> 6;
    px = g * 64u + (rem & 63u);
  } else {
    const uint32_t t = w - P.head_items, k = t / pad_px;
    c = chunk_head + k;
    px = t - k * pad_px;
  }
  uint32_t lo = 0;
  if (tile_stride) {
    lo = px / tile_stride;
  } else {
    uint32_t hi = P.n_tiles - 1;
    while (lo < hi) {
      uint32_t mid = (lo + hi + 1) >> 1;
      if (P.tiles[mid].pad_start <= px) lo = mid; else hi = mid - 1;
    }
  }
  const G::TileDev T = P.tiles[lo];
  const uint32_t q = px - T.pad_start;
  const uint32_t blk = q >> 6, in = q & 63u;
  const uint32_t lx = (blk % T.bw) * 8u + (in & 7u), ly = (blk / T.bw) * 8u + (in >> 3);
  if (lx < T.w && ly < T.h) {
    has_item = true;
    it.pxy = (T.x + lx) | ((T.y + ly) << 16);
    it.slot = c * P.n_out + (T.out_off + ly * T.w + lx);
    chunk_range(P, c, it.sample, it.sample_end);
  }
}

/* A finished sample: add it to the chunk sum in order (application.rs:448); a finished chunk goes to
 * the output (one chunk: sqrt(sum/spp), alpha 1, :451-456) or to its partial-sum slot. */
__device__ __forceinline__ void finish_sample(const KParams& P, Item& it, Vec3& sum, Vec3 rad, float scale,
                                              bool& has_item, uint32_t& n_samples, uint32_t& n_pixels) {
  sum = sum + rad;
  n_samples++;
  if (++it.sample == it.sample_end) {
    if (P.n_chunks == 1) {
      P.out[it.slot] = make_float4(sqrtf(sum.x * scale), sqrtf(sum.y * scale), sqrtf(sum.z * scale), 1.0f);
      n_pixels++;
    } else {
      P.partial[it.slot] = make_float4(sum.x, sum.y, sum.z, 0.0f);
      if (it.sample_end <= P.chunk) n_pixels++;
    }
    has_item = false;
    sum = v3(0.0f, 0.0f, 0.0f);
  }
}


__device__ __forceinline__ void flush_counts(const KParams& P, const Counts& cn) {
  atomicAdd(&P.stats[3], (unsigned long long)cn.nodes);
  atomicAdd(&P.stats[4], (unsigned long long)cn.prims);
  atomicAdd(&P.stats[5], (unsigned long long)cn.tex);
  atomicAdd(&P.stats[6], (unsigned long long)cn.walk_slots);
  atomicAdd(&P.stats[7], (unsigned long long)cn.shade_slots);
  atomicAdd(&P.stats[8], (unsigned long long)cn.prim_slots);
  atomicAdd(&P.stats[13], (unsigned long long)cn.park_slots);
  atomicAdd(&P.stats[14], (unsigned long long)cn.wait_slots);
  atomicAdd(&P.stats[16], (unsigned long long)cn.steps);
}

__device__ __forceinline__ void flush_stats(const KParams& P, uint32_t n_seg, uint32_t n_samples, uint32_t n_pixels,
                                            const Counts& cn, bool count) {
  atomicAdd(&P.stats[0], (unsigned long long)n_seg);
  atomicAdd(&P.stats[1], (unsigned long long)n_samples);
  atomicAdd(&P.stats[2], (unsigned long long)n_pixels);
  if (count) {
    atomicAdd(&P.stats[3], (unsigned long long)cn.nodes);
    atomicAdd(&P.stats[4], (unsigned long long)cn.prims);
    atomicAdd(&P.stats[5], (unsigned long long)cn.tex);
    atomicAdd(&P.stats[6], (unsigned long long)cn.walk_slots);
    atomicAdd(&P.stats[7], (unsigned long long)cn.shade_slots);
    atomicAdd(&P.stats[8], (unsigned long long)cn.prim_slots);
  }
}

#ifndef HRT_WALK_UNROLL
#define HRT_WALK_UNROLL 8
#endif
constexpr int WALK_UNROLL = HRT_WALK_UNROLL; /* node steps between two checks of the wave's exit test */
#ifndef HRT_PRIM_EVERY
#define HRT_PRIM_EVERY HRT_WALK_UNROLL
#endif
constexpr int PRIM_EVERY = HRT_PRIM_EVERY; /* node steps between two checks for batched primitive tests */
static_assert(WALK_UNROLL % PRIM_EVERY == 0, "the exit check must follow a primitive check");
#ifndef HRT_BASIC_WAVES
#define HRT_BASIC_WAVES 6
#endif
/* waves per SIMD of the sphere-scene kernel: caps its VGPRs at 512 / waves (granule 8); with the
 * scene in LDS two workgroups share a CU, so a workgroup is 128 * waves
 * threads (4 SIMDs x waves x 64 / 2). */
constexpr int BASIC_WAVES = HRT_BASIC_WAVES;
#ifndef HRT_FULL_WAVES
#define HRT_FULL_WAVES 4
#endif
constexpr int FULL_WAVES = HRT_FULL_WAVES; /* waves per SIMD of render_full_kernel (it shares the workgroup shape) */
template <bool LDS, int WAVES = BASIC_WAVES>
constexpr int basic_block_threads() { return LDS ? 128 * WAVES : 256; }


}  // namespace kern
}  // namespace hrt
