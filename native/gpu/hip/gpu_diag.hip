// MI355X (gfx950 / CDNA4) GPU health diagnostics.  See gpu_diag.h for the C ABI.  Kernels:
// HBM3E bandwidth (fill/copy/check) and the address-in-data walk over free VRAM; per-CU
// bf16 MFMA check and throughput; the MX fp8/fp4 block-scaled matrix-core check and
// throughput; the ABFT-checked GEMMs (one-wave mfma_gemm, the LDS-tiled gemm_soak and the
// 8-phase gemm_pingpong soak kernel); the burn-in loop (bf16/fp8/fp4 throughput kernels
// back to back) and pinned host<->device copies for PCIe.
//
// Design notes (CDNA4, see /opt/skills/guides):
//  * HBM phases are pure streams: 16 B per lane (global_load/store_dwordx4), 256-thread
//    blocks, 8 blocks per CU (2048 WGs >> 256 CUs) each owning one contiguous slab, 4
//    independent 16 B accesses in flight per lane so each CU keeps ~128 KiB outstanding;
//    nontemporal hints since every byte is touched exactly once per pass.  The bandwidth
//    phases run on two buffers of `bytes` each (the node agent uses 1 GiB, 4x the 256 MiB
//    Infinity Cache, so the rates are HBM rates); coverage of the whole HBM is the job of
//    the separate address-pattern walk over ~all free VRAM (walk_fill / walk_check).
//  * The MFMA test runs one v_mfma_f32_16x16x32_bf16 tile per wave per round with
//    operands in {-1,0,1} generated from a hash in registers (no memory traffic), so
//    every product sum is an exact fp32 integer and is checked element-wise against a
//    VALU recomputation.  Each wave records its physical CU (HW_REG_XCC_ID + HW_ID),
//    so a faulty matrix core is attributed to (XCC, SE, SH, CU).
//  * The throughput phase chains 4 independent accumulators per wave (dependent MFMA
//    latency hidden by 8 waves/SIMD) and verifies acc == iters * tile exactly.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "gpu_diag.h"

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;
constexpr int kUnroll = 4;

thread_local std::string g_last_error;

__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ u32x4 pattern16(uint64_t i, uint32_t seed) {
  uint32_t w = static_cast<uint32_t>(i << 2) ^ static_cast<uint32_t>(i >> 30) * 0x9e3779b9U;
  u32x4 v;
  v.x = mix32(w ^ seed);
  v.y = mix32((w + 1) ^ seed);
  v.z = mix32((w + 2) ^ seed);
  v.w = mix32((w + 3) ^ seed);
  return v;
}

// Each block streams one contiguous slab (per-block chunking keeps DRAM pages open and
// measured 5.57 TB/s copy / 6.19 TB/s read on MI355X vs 5.08 / 5.61 for a grid-stride
// interleave — tools/probes/hbm_sweep.hip, profiles/archive/hbm_sweep_r1.jsonl).
__device__ __forceinline__ void block_range(uint64_t n16, uint64_t& beg, uint64_t& end) {
  const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
  beg = static_cast<uint64_t>(blockIdx.x) * per;
  end = beg + per < n16 ? beg + per : n16;
}

__global__ __launch_bounds__(kBlock) void hbm_fill(u32x4* __restrict__ buf, uint64_t n16, uint32_t seed) {
  uint64_t beg, end;
  block_range(n16, beg, end);
  for (uint64_t b = beg + threadIdx.x; b < end; b += kBlock * kUnroll) {
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      uint64_t i = b + u * kBlock;
      if (i < end) __builtin_nontemporal_store(pattern16(i, seed), &buf[i]);
    }
  }
}

__global__ __launch_bounds__(kBlock) void hbm_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t n16) {
  uint64_t beg, end;
  block_range(n16, beg, end);
  for (uint64_t b = beg + threadIdx.x; b < end; b += kBlock * kUnroll) {
    u32x4 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      uint64_t i = b + u * kBlock;
      if (i < end) v[u] = __builtin_nontemporal_load(&src[i]);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      uint64_t i = b + u * kBlock;
      if (i < end) __builtin_nontemporal_store(v[u], &dst[i]);
    }
  }
}

__global__ __launch_bounds__(kBlock) void hbm_check(const u32x4* __restrict__ buf, uint64_t n16, uint32_t seed,
                                                    unsigned long long* __restrict__ bad,
                                                    unsigned long long* __restrict__ first_bad) {
  uint64_t beg, end;
  block_range(n16, beg, end);
  unsigned long long local_bad = 0;
  unsigned long long local_first = ~0ULL;
  for (uint64_t b = beg + threadIdx.x; b < end; b += kBlock * kUnroll) {
    u32x4 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      uint64_t i = b + u * kBlock;
      if (i < end) v[u] = __builtin_nontemporal_load(&buf[i]);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      uint64_t i = b + u * kBlock;
      if (i < end) {
        u32x4 e = pattern16(i, seed);
        int nb = (v[u].x != e.x) + (v[u].y != e.y) + (v[u].z != e.z) + (v[u].w != e.w);
        if (nb) {
          local_bad += nb;
          local_first = std::min<unsigned long long>(local_first, i * 4);
        }
      }
    }
  }
  if (local_bad) {
    atomicAdd(bad, local_bad);
    atomicMin(first_bad, local_first);
  }
}

// ---------------------------------------------------------------------------
// HBM walk (bgc_diag_hbm_walk): every 64-bit word holds its own device address ^ key.
// A stuck bit, a weak cell or a write that decodes to the wrong row/bank/stack shows up
// at verify time as a word whose content is not its address.  The inverse pass is the
// same kernel with ~key, so every bit is checked at 0 and at 1.

__device__ __forceinline__ u32x4 walk_value(const u32x4* p, uint64_t key) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint64_t w0 = a ^ key, w1 = (a + 8) ^ key;
  u32x4 v;
  v.x = static_cast<uint32_t>(w0);
  v.y = static_cast<uint32_t>(w0 >> 32);
  v.z = static_cast<uint32_t>(w1);
  v.w = static_cast<uint32_t>(w1 >> 32);
  return v;
}

__global__ __launch_bounds__(kBlock) void walk_fill(u32x4* __restrict__ buf, uint64_t n16, uint64_t key) {
  uint64_t beg, end;
  block_range(n16, beg, end);
  for (uint64_t b = beg + threadIdx.x; b < end; b += kBlock * kUnroll) {
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const uint64_t i = b + u * kBlock;
      if (i < end) __builtin_nontemporal_store(walk_value(&buf[i], key), &buf[i]);
    }
  }
}

__global__ __launch_bounds__(kBlock) void walk_check(const u32x4* __restrict__ buf, uint64_t n16, uint64_t key,
                                                     unsigned long long* __restrict__ bad,
                                                     unsigned long long* __restrict__ first_bad_addr) {
  uint64_t beg, end;
  block_range(n16, beg, end);
  unsigned long long local_bad = 0, local_first = ~0ULL;
  for (uint64_t b = beg + threadIdx.x; b < end; b += kBlock * kUnroll) {
    u32x4 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const uint64_t i = b + u * kBlock;
      if (i < end) v[u] = __builtin_nontemporal_load(&buf[i]);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const uint64_t i = b + u * kBlock;
      if (i < end) {
        const u32x4 e = walk_value(&buf[i], key);
        const bool b0 = v[u].x != e.x || v[u].y != e.y, b1 = v[u].z != e.z || v[u].w != e.w;
        if (b0 || b1) {
          local_bad += static_cast<unsigned long long>(b0) + static_cast<unsigned long long>(b1);
          const uint64_t a = reinterpret_cast<uint64_t>(&buf[i]) + (b0 ? 0 : 8);
          local_first = std::min<unsigned long long>(local_first, a);
        }
      }
    }
  }
  if (local_bad) {
    atomicAdd(bad, local_bad);
    atomicMin(first_bad_addr, local_first);
  }
}

// ---------------------------------------------------------------------------
// MFMA

__device__ __forceinline__ int operand(uint32_t seed, uint32_t tile, int r, int c, uint32_t which) {
  uint32_t h = mix32(seed ^ mix32(tile * 0x9e3779b9U + which) ^ static_cast<uint32_t>(r * 64 + c));
  return static_cast<int>(h % 3u) - 1;
}

__device__ __forceinline__ uint32_t cu_key() {
  uint32_t xcc, hwid;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
  uint32_t cu = (hwid >> 8) & 0xF;
  uint32_t sh = (hwid >> 12) & 0x1;
  uint32_t se = (hwid >> 13) & 0x7;
  return ((xcc & 0x7) << 8) | (se << 5) | (sh << 4) | cu;
}

// One wave = one 16x16x32 tile per round. A is 16x32, B is 32x16.
__global__ __launch_bounds__(kBlock) void mfma_check(uint32_t seed, int rounds, unsigned* __restrict__ cu_tiles,
                                                     unsigned* __restrict__ cu_bad) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = (blockIdx.x * (kBlock / 64)) + (threadIdx.x >> 6);
  const uint32_t key = cu_key();
  unsigned bad = 0;
  for (int r = 0; r < rounds; ++r) {
    const uint32_t tile = wave * static_cast<uint32_t>(rounds) + static_cast<uint32_t>(r);
    bf16x8 a, b;
    const int row = lane & 15;
    const int kb = 8 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a[j] = static_cast<__bf16>(static_cast<float>(operand(seed, tile, row, kb + j, 0xA)));
      b[j] = static_cast<__bf16>(static_cast<float>(operand(seed, tile, kb + j, row, 0xB)));
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    const int col = lane & 15;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int orow = (lane >> 4) * 4 + i;
      int expect = 0;
      for (int k = 0; k < 32; ++k) expect += operand(seed, tile, orow, k, 0xA) * operand(seed, tile, k, col, 0xB);
      bad += (acc[i] != static_cast<float>(expect));
    }
  }
  // one atomic per wave (lane 0 after a wave reduction)
  for (int off = 32; off > 0; off >>= 1) bad += __shfl_down(bad, off, 64);
  if (lane == 0) {
    atomicAdd(&cu_tiles[key], static_cast<unsigned>(rounds));
    if (bad) atomicAdd(&cu_bad[key], bad);
  }
}

// Each wave also times itself on the 100 MHz constant clock and adds its duration to
// its XCC's bin, so a slow (throttled / degraded) XCC shows up as an imbalance even when
// the whole-chip rate still clears its floor.
__global__ __launch_bounds__(kBlock) void mfma_throughput(uint32_t seed, int iters, unsigned* __restrict__ fails,
                                                          unsigned long long* __restrict__ xcc_ticks,
                                                          unsigned* __restrict__ xcc_waves) {
  const uint64_t t_start = wall_clock64();
  const int lane = threadIdx.x & 63;
  const uint32_t tile = (blockIdx.x * (kBlock / 64)) + (threadIdx.x >> 6);
  const int row = lane & 15;
  const int kb = 8 * (lane >> 4);
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = static_cast<__bf16>(static_cast<float>(operand(seed, tile, row, kb + j, 0xA)));
    b[j] = static_cast<__bf16>(static_cast<float>(operand(seed, tile, kb + j, row, 0xB)));
  }
  // Distinct initial values keep the compiler from merging the four chains.
  f32x4 acc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = f32x4{float(c), float(c), float(c), float(c)};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[c], 0, 0, 0);
  }
  const int col = lane & 15;
  unsigned bad = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int orow = (lane >> 4) * 4 + i;
    int expect = 0;
    for (int k = 0; k < 32; ++k) expect += operand(seed, tile, orow, k, 0xA) * operand(seed, tile, k, col, 0xB);
    const float e = static_cast<float>(expect) * static_cast<float>(iters);
#pragma unroll
    for (int c = 0; c < 4; ++c) bad += (acc[c][i] != e + float(c));
  }
  for (int off = 32; off > 0; off >>= 1) bad += __shfl_down(bad, off, 64);
  const uint64_t t_end = wall_clock64();  // after the accumulators were consumed above
  if (lane == 0) {
    if (bad) atomicAdd(fails, bad);
    const uint32_t xcc = (cu_key() >> 8) & 7;
    atomicAdd(&xcc_ticks[xcc], static_cast<unsigned long long>(t_end - t_start));
    atomicAdd(&xcc_waves[xcc], 1u);
  }
}

// ---------------------------------------------------------------------------
// Low-precision (MX block-scaled) matrix cores: v_mfma_scale_f32_16x16x128_f8f6f4.
// Lane l holds 32 K-elements of A row (l & 15) and of B column (l & 15) from lane group
// g = l >> 4, plus one E8M0 scale byte for (its row or column, block g) of the 4 K-blocks
// of 32.  A and B are laid out alike, so A element (g, j) always meets B element (g, j);
// which block, hence which scale, an element belongs to is lowp_block().  The exact
// result is sum_blk 2^(sa(r, blk) + sb(c, blk)) * sum_{(g, j) in blk} a(r, g, j) b(c, g, j).
// Operands in {-1, 0, 1} and scales in {1/2, 1, 2} keep every product and sum exact.
// kFmt: 0 = fp8 e4m3 (OCP), 4 = fp4 e2m1 (two per byte; 16 of the 32 operand bytes).
typedef int i32x8 __attribute__((ext_vector_type(8)));

template <int kFmt>
__device__ __forceinline__ uint32_t lowp_code(int v) {
  if (kFmt == 0) return v > 0 ? 0x38u : (v < 0 ? 0xB8u : 0u);  // e4m3: +-1.0 = 0 0111 000
  return v > 0 ? 0x2u : (v < 0 ? 0xAu : 0u);                  // e2m1: +-1.0 = 0 01 0
}

// 32 operands of one lane (row or column `rc`, block `g`) packed for the MFMA
template <int kFmt>
__device__ __forceinline__ i32x8 lowp_pack(uint32_t seed, uint32_t tile, int rc, int g, uint32_t which) {
  i32x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const uint32_t c = lowp_code<kFmt>(operand(seed, tile, rc, 32 * g + j, which));
    if (kFmt == 0) {
      v[j >> 2] |= static_cast<int>(c << (8 * (j & 3)));
    } else {
      v[j >> 3] |= static_cast<int>(c << (4 * (j & 7)));
    }
  }
  return v;
}

// The scale block (= the lane group whose scale byte applies) of element j of lane group g,
// measured on the MI355X with tools/probes/mx_scale_layout.hip (profiles/mx_lowp_r3/):
//  * fp4: a lane group's 32 elements are K 32g..32g+31, one block, its own scale;
//  * fp8: elements 0-15 are K 16g..16g+15 and 16-31 are K 64+16g.., so they fall in
//    blocks g/2 and 2+g/2, scaled by lane groups g/2 and 2+g/2.
template <int kFmt>
__device__ __forceinline__ int lowp_block(int g, int j) {
  return kFmt == 0 ? (g >> 1) + 2 * (j >> 4) : g;
}

// scale exponent in {-1, 0, 1} for (row or column, block); 0 when unscaled
__device__ __forceinline__ int lowp_exp(uint32_t seed, uint32_t tile, int rc, int g, uint32_t which, bool scaled) {
  return scaled ? operand(seed ^ 0x5ca1e, tile, rc, g, which) : 0;
}

template <int kFmt>
__device__ __forceinline__ f32x4 lowp_mfma(i32x8 a, i32x8 b, f32x4 acc, int sa, int sb) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, kFmt, kFmt, 0, 127 + sa, 0, 127 + sb);
}

template <int kFmt>
__global__ __launch_bounds__(kBlock) void mfma_lowp_check(uint32_t seed, int rounds, int scaled,
                                                          unsigned* __restrict__ cu_tiles,
                                                          unsigned* __restrict__ cu_bad) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = (blockIdx.x * (kBlock / 64)) + (threadIdx.x >> 6);
  const uint32_t key = cu_key();
  const int rc = lane & 15, g = lane >> 4;
  unsigned bad = 0;
  for (int r = 0; r < rounds; ++r) {
    const uint32_t tile = wave * static_cast<uint32_t>(rounds) + static_cast<uint32_t>(r);
    const i32x8 a = lowp_pack<kFmt>(seed, tile, rc, g, 0xA);
    const i32x8 b = lowp_pack<kFmt>(seed, tile, rc, g, 0xB);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = lowp_mfma<kFmt>(a, b, acc, lowp_exp(seed, tile, rc, g, 0xA, scaled), lowp_exp(seed, tile, rc, g, 0xB, scaled));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int orow = 4 * g + i;  // the C/D map of every 16x16 MFMA: column lane & 15, row 4 (lane >> 4) + i
      int dot[4] = {0, 0, 0, 0};  // per scale block
      for (int gg = 0; gg < 4; ++gg) {
        for (int j = 0; j < 32; ++j) {
          dot[lowp_block<kFmt>(gg, j)] +=
              operand(seed, tile, orow, 32 * gg + j, 0xA) * operand(seed, tile, rc, 32 * gg + j, 0xB);
        }
      }
      float expect = 0.f;
      for (int blk = 0; blk < 4; ++blk) {
        const int e = lowp_exp(seed, tile, orow, blk, 0xA, scaled) + lowp_exp(seed, tile, rc, blk, 0xB, scaled);
        expect += ldexpf(static_cast<float>(dot[blk]), e);
      }
      bad += (acc[i] != expect);
    }
  }
  for (int off = 32; off > 0; off >>= 1) bad += __shfl_down(bad, off, 64);
  if (lane == 0) {
    atomicAdd(&cu_tiles[key], static_cast<unsigned>(rounds));
    if (bad) atomicAdd(&cu_bad[key], bad);
  }
}

// Rate: 4 independent accumulator chains per wave, unit scales, acc == iters * tile + c
template <int kFmt>
__global__ __launch_bounds__(kBlock) void mfma_lowp_throughput(uint32_t seed, int iters, unsigned* __restrict__ fails) {
  const int lane = threadIdx.x & 63;
  const uint32_t tile = (blockIdx.x * (kBlock / 64)) + (threadIdx.x >> 6);
  const int rc = lane & 15, g = lane >> 4;
  const i32x8 a = lowp_pack<kFmt>(seed, tile, rc, g, 0xA);
  const i32x8 b = lowp_pack<kFmt>(seed, tile, rc, g, 0xB);
  f32x4 acc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = f32x4{float(c), float(c), float(c), float(c)};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = lowp_mfma<kFmt>(a, b, acc[c], 0, 0);
  }
  unsigned bad = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int orow = 4 * g + i;
    int expect = 0;
    for (int k = 0; k < 128; ++k) expect += operand(seed, tile, orow, k, 0xA) * operand(seed, tile, rc, k, 0xB);
    const float e = static_cast<float>(expect) * static_cast<float>(iters);
#pragma unroll
    for (int c = 0; c < 4; ++c) bad += (acc[c][i] != e + float(c));
  }
  for (int off = 32; off > 0; off >>= 1) bad += __shfl_down(bad, off, 64);
  if (lane == 0 && bad) atomicAdd(fails, bad);
}

// MX GEMM on caller operands, for the host cross-check of the block-scaled path against an
// independent decode (PyTorch): C[m, n] = sum_k a(m, k) 2^(sa(m, k/32) - 127) *
// b(n, k) 2^(sb(n, k/32) - 127).  A is M x K codes (fp8: one byte each; fp4: two per byte,
// element 2i in the low nibble), Bt is N x K alike, the E8M0 scales are M x K/32 and
// N x K/32 bytes.  One wave per 16x16 output tile, K consumed 128 at a time; each lane loads
// its operands straight from memory in the MFMA's own layout (lowp_block above): fp8 lane
// group g holds K 16g..16g+15 then 64+16g..64+16g+15, fp4 lane group g holds K 32g..32g+31.
template <int kFmt>
__device__ __forceinline__ i32x8 lowp_load(const uint8_t* __restrict__ X, int row, int K, int k0, int g) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  i32x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
  if (kFmt == 0) {
    const uint8_t* p = X + static_cast<size_t>(row) * K + k0 + 16 * g;
    const i32x4 lo = *reinterpret_cast<const i32x4*>(p);
    const i32x4 hi = *reinterpret_cast<const i32x4*>(p + 64);
    v = i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  } else {
    const i32x4 q = *reinterpret_cast<const i32x4*>(X + static_cast<size_t>(row) * (K / 2) + (k0 + 32 * g) / 2);
    v = i32x8{q[0], q[1], q[2], q[3], 0, 0, 0, 0};
  }
  return v;
}

template <int kFmt>
__global__ __launch_bounds__(64) void mx_gemm(const uint8_t* __restrict__ A, const uint8_t* __restrict__ sA,
                                              const uint8_t* __restrict__ Bt, const uint8_t* __restrict__ sB,
                                              float* __restrict__ C, int M, int N, int K) {
  const int lane = threadIdx.x, rc = lane & 15, g = lane >> 4;
  const int tiles_n = N / 16;
  const int m0 = (static_cast<int>(blockIdx.x) / tiles_n) * 16, n0 = (static_cast<int>(blockIdx.x) % tiles_n) * 16;
  const int kb = K / 32;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += 128) {
    const i32x8 a = lowp_load<kFmt>(A, m0 + rc, K, k0, g);
    const i32x8 b = lowp_load<kFmt>(Bt, n0 + rc, K, k0, g);
    const int sa = sA[static_cast<size_t>(m0 + rc) * kb + k0 / 32 + g];  // this lane's (row, block g) scale
    const int sb = sB[static_cast<size_t>(n0 + rc) * kb + k0 / 32 + g];
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, kFmt, kFmt, 0, sa, 0, sb);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) C[static_cast<size_t>(m0 + 4 * g + i) * N + n0 + rc] = acc[i];
}

// Plain MFMA GEMM for the host cross-check: C[M,N] (fp32) = A[M,K] * B[K,N] (bf16,
// row-major).  One wave per 16x16 output tile, K consumed 32 at a time by
// v_mfma_f32_16x16x32_bf16 with the same operand layout as the tests above: lane l
// holds A row (l & 15) / B column (l & 15), k = 8 * (l >> 4) + j; the result lane l
// holds column (l & 15), rows 4 * (l >> 4) + i.
__global__ __launch_bounds__(64) void mfma_gemm(const __bf16* __restrict__ A, const __bf16* __restrict__ B,
                                                float* __restrict__ C, int M, int N, int K) {
  const int lane = threadIdx.x;
  const int tm = blockIdx.y * 16, tn = blockIdx.x * 16;
  const int rc = lane & 15, kb = 8 * (lane >> 4);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += 32) {
    bf16x8 a, b;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a[j] = A[static_cast<size_t>(tm + rc) * K + k0 + kb + j];
      b[j] = B[static_cast<size_t>(k0 + kb + j) * N + tn + rc];
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) C[static_cast<size_t>(tm + 4 * (lane >> 4) + i) * N + tn + rc] = acc[i];
  (void)M;
}


// ---------------------------------------------------------------------------
// GEMM soak: an LDS-tiled bf16 MFMA GEMM run back to back, verified by checksums.
//
// Unlike mfma_throughput (operands in registers), this exercises the whole matrix path a
// training step uses: HBM -> LDS by global_load_lds (16 B per lane, no VGPR round trip),
// LDS -> VGPR fragment reads, MFMA, and C written back to HBM.
//  * Tile 128x128x64, 4 waves (2x2, 64x64 per wave = 4x4 accumulators of 16x16), two LDS
//    buffers (2 x 32 KiB): tile k+1 streams in while tile k is multiplied; one
//    vmcnt(0) + barrier per K-step.  64 KiB per block -> 2 blocks per CU.
//  * LDS image [128 rows][8 chunks of 16 B] with chunk p of row r holding source chunk
//    p ^ (r & 7): the 16 rows a fragment read touches land on distinct 16-B slots of the
//    bank row (linear rows 128 B apart would stack 8 deep).  glds writes lane-linear LDS,
//    so the swizzle is applied to the GLOBAL source address.
//  * B is given transposed (Bt[N][K]) so both operands are K-contiguous.
//  * Blocks are remapped XCD-aware (bijective for any grid) and grouped 8 tile-rows at a
//    time so the tiles sharing A rows / B columns run on one XCD's L2.
// Verification (ABFT): operands in {-1, 0, 1} make every C element an exact integer, so
// C's row sums must equal A * (B 1) and its column sums (1^T A) * B, both computed with
// integer kernels on a separate path; any wrong element shows in its row and its column.
constexpr int kSoakBK = 64;

__device__ __forceinline__ bf16x8 soak_frag(const char* base, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(base + row * 128 + ((chunk ^ (row & 7)) << 4));
}

// BM x BN tile, WM x WN waves (each wave (BM/WM) x (BN/WN) outputs as 16x16 MFMA tiles).
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN, (BM * BN >= 256 * 256) ? 1 : 2) void gemm_soak(
    const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, float* __restrict__ C, int M, int N, int K) {
  constexpr int kWaves = WM * WN;
  constexpr int kMI = BM / WM / 16, kNI = BN / WN / 16;
  constexpr int kA = BM * kSoakBK * 2, kB = BN * kSoakBK * 2;  // bytes per stage
  constexpr int kAInstr = BM / 8 / kWaves, kBInstr = BN / 8 / kWaves;  // 8 rows of 128 B per wave-instruction
  static_assert(BM % (8 * kWaves) == 0 && BN % (8 * kWaves) == 0, "tile rows must split over the waves");
  __shared__ __attribute__((aligned(16))) char lds[2 * (kA + kB)];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WN, wc = wid % WN;
  // XCD-aware bijective remap: consecutive ids of one XCD get consecutive tiles
  const int nwg = static_cast<int>(gridDim.x), orig = static_cast<int>(blockIdx.x);
  const int xcd = orig % 8, q = nwg / 8, r = nwg % 8;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  // grouped ordering: 8 tile-rows share each B column tile in L2
  const int tiles_m = M / BM, tiles_n = N / BN, group = 8;
  const int per_group = group * tiles_n;
  const int first_m = (wgid / per_group) * group;
  const int gsize = min(tiles_m - first_m, group);
  const int tm = first_m + (wgid % per_group) % gsize;
  const int tn = (wgid % per_group) / gsize;

  auto stage = [&](int buf, int k0) {
    char* a_l = lds + buf * (kA + kB);
    char* b_l = a_l + kA;
#pragma unroll
    for (int i = 0; i < kAInstr; ++i) {
      const int row0 = (wid * kAInstr + i) * 8;
      const int row = row0 + (lane >> 3);
      const int chunk = (lane & 7) ^ (row & 7);  // source chunk for LDS slot (lane & 7)
      const __bf16* g = A + static_cast<size_t>(tm * BM + row) * K + k0 + chunk * 8;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                       (__attribute__((address_space(3))) void*)(a_l + row0 * 128), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < kBInstr; ++i) {
      const int row0 = (wid * kBInstr + i) * 8;
      const int row = row0 + (lane >> 3);
      const int chunk = (lane & 7) ^ (row & 7);
      const __bf16* g = Bt + static_cast<size_t>(tn * BN + row) * K + k0 + chunk * 8;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                       (__attribute__((address_space(3))) void*)(b_l + row0 * 128), 16, 0, 0);
    }
  };

  f32x4 acc[kMI][kNI];
#pragma unroll
  for (int mi = 0; mi < kMI; ++mi)
#pragma unroll
    for (int ni = 0; ni < kNI; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int kt_n = K / kSoakBK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < kt_n; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < kt_n) stage(buf ^ 1, (kt + 1) * kSoakBK);  // streams in under this tile's MFMAs
    const char* a_l = lds + buf * (kA + kB);
    const char* b_l = a_l + kA;
#pragma unroll
    for (int s = 0; s < 2; ++s) {  // two K=32 MFMA steps per 64-deep tile
      bf16x8 af[kMI], bfr[kNI];
#pragma unroll
      for (int mi = 0; mi < kMI; ++mi) af[mi] = soak_frag(a_l, wr * (BM / WM) + mi * 16 + (lane & 15), s * 4 + (lane >> 4));
#pragma unroll
      for (int ni = 0; ni < kNI; ++ni) bfr[ni] = soak_frag(b_l, wc * (BN / WN) + ni * 16 + (lane & 15), s * 4 + (lane >> 4));
#pragma unroll
      for (int mi = 0; mi < kMI; ++mi)
#pragma unroll
        for (int ni = 0; ni < kNI; ++ni) acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next tile has landed ...
    __syncthreads();                                   // ... and nobody still reads this one
  }
#pragma unroll
  for (int mi = 0; mi < kMI; ++mi)
#pragma unroll
    for (int ni = 0; ni < kNI; ++ni)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const size_t row = static_cast<size_t>(tm * BM + wr * (BM / WM) + mi * 16 + (lane >> 4) * 4 + j);
        C[row * N + tn * BN + wc * (BN / WN) + ni * 16 + (lane & 15)] = acc[mi][ni][j];
      }
}

// ---------------------------------------------------------------------------
// 256x256 ping-pong GEMM: the soak's kernel whenever K is a multiple of 128.
//
// The 2-buffer kernel above drains every K-tile's loads (vmcnt(0) + barrier) one tile
// after issuing them; with one 512-thread block per CU a tile's 64 MFMAs per wave
// (~0.9 us per SIMD) do not cover an HBM/L2 fetch under full load, and the matrix pipe
// sat idle 42 % of the time (profiles/archive/gemm_soak_r2/pmc_soak_8192.json).  This kernel
// keeps the same LDS budget (two K-tiles, 128 KiB) but manages it in eight 16 KiB
// half-tiles (A rows 0-127 / 128-255, Bt rows 0-127 / 128-255 of each K-tile):
//
//  * Two wave groups, waves 0-3 (output rows 0-127) and 4-7 (rows 128-255): each SIMD
//    hosts one wave of each.  Group 1 runs one s_barrier behind group 0, so between any
//    two barriers one wave of a SIMD issues its 16 MFMAs while its partner issues LDS
//    fragment reads and global->LDS loads — matrix beside memory, never matrix beside
//    matrix.
//  * A phase is one C quadrant of the wave's 128x64 output (4x2 tiles of 16x16, K=64):
//    16 v_mfma_f32_16x16x32_bf16.  Eight phases = two K-tiles per loop iteration.
//    Fragments: all of the wave's B (64 columns) and half its A at phase 0, the other A
//    half at phase 2 (192 VGPRs: 128 accumulator, 32 A, 32 B).
//  * Two half-tile loads in every odd phase (the even phases carry all the fragment
//    reads), each into a half last read at least two barriers earlier (B halves are read
//    only in the first phase of a K-tile, A halves in the first and third).  Waits are
//    counted, vmcnt(4) at phases 3 and 7 (each half-tile is 2 glds per thread), and a
//    half is first read one phase after the wait that retires it; loads stay in flight
//    across the barriers.  (kSched 0, BGC_SOAK_KERNEL=pingpong0: the first schedule, one
//    half-tile in every phase.)
//  * Staging past the last K-tile re-reads the last tile into a buffer nobody reads
//    again, so the vmcnt counts never change; the block drains (vmcnt(0)) before its
//    epilogue.
constexpr int kPPHalf = 128 * 128;  // one half-tile image: 128 rows x 64 k x 2 B

__device__ __forceinline__ void pp_stage(char* lds, int half, const __bf16* __restrict__ src, int K, int row_base, int k0,
                                         int wid, int lane) {
  char* dst = lds + half * kPPHalf;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row0 = (i * 8 + wid) * 8;  // 8 rows of 128 B per wave-instruction
    const int row = row0 + (lane >> 3);
    const int chunk = (lane & 7) ^ (row & 7);  // LDS slot (lane & 7) holds source chunk ^ swizzle
    const __bf16* g = src + static_cast<size_t>(row_base + row) * K + k0 + chunk * 8;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)(dst + row0 * 128), 16, 0, 0);
  }
}

__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int kSched>  // 0: a half-tile load in every phase; 2: two in every odd phase
__global__ __launch_bounds__(512, 1) void gemm_pingpong(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt,
                                                        float* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char lds[8 * kPPHalf];  // [buf][A_top, A_bot, B_left, B_right]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;  // wave group = output row half
  // XCD-aware bijective remap + 8 tile-rows grouped per B column tile (as gemm_soak)
  const int nwg = static_cast<int>(gridDim.x), orig = static_cast<int>(blockIdx.x);
  const int xcd = orig % 8, q = nwg / 8, r = nwg % 8;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  const int tiles_m = M / 256, tiles_n = N / 256, group = 8;
  const int per_group = group * tiles_n;
  const int first_m = (wgid / per_group) * group;
  const int gsize = min(tiles_m - first_m, group);
  const int tm = first_m + (wgid % per_group) % gsize;
  const int tn = (wgid % per_group) / gsize;
  const int kt_n = K / kSoakBK;
  const int a_row = tm * 256, b_row = tn * 256;
  auto kofs = [&](int t) { return min(t, kt_n - 1) * kSoakBK; };
  // half-tile images of buffer b: A_top 4b, A_bot 4b+1, B_left 4b+2, B_right 4b+3
  auto stage = [&](int half, int t) {
    const int h = half & 3;
    if (h < 2) pp_stage(lds, half, A, K, a_row + h * 128, kofs(t), wid, lane);
    else pp_stage(lds, half, Bt, K, b_row + (h - 2) * 128, kofs(t), wid, lane);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2], bfr[4][2];

  // prologue: K-tile 0 into buffer 0, K-tile 1's B halves into buffer 1
  stage(0, 0);
  stage(1, 0);
  stage(2, 0);
  stage(3, 0);
  stage(6, 1);
  stage(7, 1);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  pp_barrier();
  if (wr == 1) pp_barrier();  // the stagger: group 1 runs one barrier behind

  const int a_half = wr;            // A image this wave reads (per buffer)
  const int b_half = 2 + (wc >> 1);  // Bt image
  const int b_row0 = (wc & 1) * 64;  // first of the wave's 64 Bt rows inside that image

  for (int it = 0; it < kt_n / 2; ++it) {
    const int t_odd = 2 * it + 1, t_next = 2 * it + 2, t_next_odd = 2 * it + 3;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const char* buf = lds + (p >> 2) * 4 * kPPHalf;
      if ((p & 3) == 0) {  // all of B, rows 0-63 of A
        const char* bi = buf + b_half * kPPHalf;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) bfr[ni][ks] = soak_frag(bi, b_row0 + ni * 16 + (lane & 15), ks * 4 + (lane >> 4));
      }
      if ((p & 1) == 0) {  // phases 0/2 (4/6): the A half this quadrant pair needs
        const char* ai = buf + a_half * kPPHalf;
        const int m0 = (p & 2) ? 64 : 0;
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) af[mi][ks] = soak_frag(ai, m0 + mi * 16 + (lane & 15), ks * 4 + (lane >> 4));
      }
      if constexpr (kSched == 2) {
        // All fragment reads happen in the even phases (16 at 0/4, 8 at 2/6; at four
        // reading waves per CU, 16 take the partner's whole MFMA interval), so the loads
        // go to the odd phases, two half-tiles each.  Same halves; each is still reloaded
        // >= 2 barriers after its last read, and vmcnt(4) at phases 3/7 retires phases
        // 1/5 (profiles/gemm_soak_r3/: +3-7 % at 4096^3, +0.5 % at 8192^3)
        switch (p) {
          case 1: stage(4, t_odd); stage(5, t_odd); break;           // buffer 1 A (read at phase 4)
          case 3: stage(2, t_next); stage(3, t_next); break;         // buffer 0 B (last read at phase 0)
          case 5: stage(0, t_next); stage(1, t_next); break;         // buffer 0 A (last read at phase 2)
          case 7: stage(6, t_next_odd); stage(7, t_next_odd); break; // buffer 1 B (last read at phase 4)
          default: break;
        }
      } else {
        switch (p) {  // one half-tile per phase, each into a half nobody reads any more
          case 0: stage(4, t_odd); break;      // buffer 1 A_top (read at phase 4)
          case 1: stage(5, t_odd); break;      // buffer 1 A_bot
          case 2: stage(2, t_next); break;     // buffer 0 B_left (last read at phase 0)
          case 3: stage(3, t_next); break;     // buffer 0 B_right
          case 4: stage(0, t_next); break;     // buffer 0 A_top (last read at phase 2)
          case 5: stage(1, t_next); break;     // buffer 0 A_bot
          case 6: stage(6, t_next_odd); break; // buffer 1 B_left (last read at phase 4)
          default: stage(7, t_next_odd); break;
        }
      }
      if ((p & 3) == 3) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // retires everything through phase p-2
      pp_barrier();
      __builtin_amdgcn_s_setprio(1);
      const int mh = (p >> 1) & 1, nh = p & 1;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
            acc[mh * 4 + mi][nh * 2 + ni] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi][ks], bfr[nh * 2 + ni][ks], acc[mh * 4 + mi][nh * 2 + ni], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      pp_barrier();
    }
  }
  if (wr == 0) pp_barrier();  // matches group 1's extra barrier
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the block
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const size_t row = static_cast<size_t>(a_row + wr * 128 + mi * 16 + (lane >> 4) * 4 + j);
        C[row * N + b_row + wc * 64 + ni * 16 + (lane & 15)] = acc[mi][ni][j];
      }
}

// X[rows][cols] = hash-derived values in {-1, 0, 1} (exact in bf16)
__global__ __launch_bounds__(kBlock) void soak_fill(__bf16* __restrict__ X, uint64_t n, uint32_t seed) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * kBlock) {
    const uint32_t h = mix32(static_cast<uint32_t>(i) ^ mix32(static_cast<uint32_t>(i >> 32) + seed));
    X[i] = static_cast<__bf16>(static_cast<float>(static_cast<int>(h % 3u) - 1));
  }
}

// out[c] += sum over a 64-row slab of X[r][c]  (column sums, integer)
__global__ __launch_bounds__(kBlock) void soak_colsum(const __bf16* __restrict__ X, int rows, int cols, int* __restrict__ out) {
  const int c = blockIdx.x * kBlock + threadIdx.x;
  if (c >= cols) return;
  const int r0 = blockIdx.y * 64, r1 = min(rows, r0 + 64);
  int s = 0;
  for (int r = r0; r < r1; ++r) s += static_cast<int>(static_cast<float>(X[static_cast<size_t>(r) * cols + c]));
  atomicAdd(&out[c], s);
}

// out[r] = sum_k X[r][k] * v[k]  (one block per row, integer)
__global__ __launch_bounds__(kBlock) void soak_rowdot(const __bf16* __restrict__ X, int cols, const int* __restrict__ v,
                                                      long long* __restrict__ out) {
  __shared__ long long part[kBlock];
  const size_t base = static_cast<size_t>(blockIdx.x) * cols;
  long long s = 0;
  for (int k = threadIdx.x; k < cols; k += kBlock) s += static_cast<long long>(static_cast<float>(X[base + k])) * v[k];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if (static_cast<int>(threadIdx.x) < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = part[0];
}

// row sums (one block per row) and column sums (atomics over 64-row slabs) of C, as exact integers
__global__ __launch_bounds__(kBlock) void soak_c_rowsum(const float* __restrict__ C, int cols, long long* __restrict__ out) {
  __shared__ long long part[kBlock];
  const size_t base = static_cast<size_t>(blockIdx.x) * cols;
  long long s = 0;
  for (int k = threadIdx.x; k < cols; k += kBlock) s += llrintf(C[base + k]);
  part[threadIdx.x] = s;
  __syncthreads();
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if (static_cast<int>(threadIdx.x) < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = part[0];
}

__global__ __launch_bounds__(kBlock) void soak_c_colsum(const float* __restrict__ C, int rows, int cols,
                                                        unsigned long long* __restrict__ out) {
  const int c = blockIdx.x * kBlock + threadIdx.x;
  if (c >= cols) return;
  const int r0 = blockIdx.y * 64, r1 = min(rows, r0 + 64);
  long long s = 0;
  for (int r = r0; r < r1; ++r) s += llrintf(C[static_cast<size_t>(r) * cols + c]);
  atomicAdd(&out[c], static_cast<unsigned long long>(s));  // two's complement: signed sums add correctly
}

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      g_last_error = std::string(#expr) + ": " + hipGetErrorString(_e);                 \
      return 1;                                                                         \
    }                                                                                   \
  } while (0)

int cu_count(int device) {
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n <= 0) n = 256;
  return n;
}

struct DeviceBuffer {
  void* p = nullptr;
  ~DeviceBuffer() {
    if (p) (void)hipFree(p);
  }
};

struct Events {
  hipEvent_t a = nullptr, b = nullptr;
  ~Events() {
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
  }
};

struct HostBuffer {  // pinned: DMA straight from/to it, no staging copy
  void* p = nullptr;
  ~HostBuffer() {
    if (p) (void)hipHostFree(p);
  }
};

struct Streams {
  hipStream_t a = nullptr, b = nullptr;
  ~Streams() {
    if (a) (void)hipStreamDestroy(a);
    if (b) (void)hipStreamDestroy(b);
  }
};

struct Chunks {  // the HBM walk's allocations, freed on every exit path
  std::vector<std::pair<void*, uint64_t>> v;
  ~Chunks() {
    for (auto& c : v) (void)hipFree(c.first);
  }
};

// 256x256 tiles (8 waves, 128 KiB LDS, 1 block/CU) when the shape divides; else 128x128
bool soak_big_tile(int m, int n) {
  const char* tile_env = std::getenv("BGC_SOAK_TILE");
  return (m % 256 == 0 && n % 256 == 0) && !(tile_env && std::string(tile_env) == "128");
}

// BGC_SOAK_KERNEL=2buf keeps the double-buffered kernel for A/B runs
bool soak_pingpong(bool big, int k) {
  const char* kern = std::getenv("BGC_SOAK_KERNEL");
  return big && k % (2 * kSoakBK) == 0 && !(kern && std::string(kern) == "2buf");
}

void launch_soak_gemm(bool big, const void* a, const void* bt, void* c, int m, int n, int k, hipStream_t s) {
  if (soak_pingpong(big, k)) {
    // BGC_SOAK_KERNEL=pingpong0: the first schedule (one half-tile load in every phase)
    const char* kern = std::getenv("BGC_SOAK_KERNEL");
    if (kern && std::string(kern) == "pingpong0") {
      hipLaunchKernelGGL(gemm_pingpong<0>, dim3((m / 256) * (n / 256)), dim3(512), 0, s,
                         static_cast<const __bf16*>(a), static_cast<const __bf16*>(bt), static_cast<float*>(c), m, n, k);
    } else {
      hipLaunchKernelGGL(gemm_pingpong<2>, dim3((m / 256) * (n / 256)), dim3(512), 0, s,
                         static_cast<const __bf16*>(a), static_cast<const __bf16*>(bt), static_cast<float*>(c), m, n, k);
    }
  } else if (big) {
    hipLaunchKernelGGL((gemm_soak<256, 256, 2, 4>), dim3((m / 256) * (n / 256)), dim3(512), 0, s,
                       static_cast<const __bf16*>(a), static_cast<const __bf16*>(bt), static_cast<float*>(c), m, n, k);
  } else {
    hipLaunchKernelGGL((gemm_soak<128, 128, 2, 2>), dim3((m / 128) * (n / 128)), dim3(256), 0, s,
                       static_cast<const __bf16*>(a), static_cast<const __bf16*>(bt), static_cast<float*>(c), m, n, k);
  }
}

bool soak_shape_ok(int m, int n, int k) {
  return m >= 128 && n >= 128 && k >= kSoakBK && m % 128 == 0 && n % 128 == 0 && k % kSoakBK == 0 && m <= 32768 &&
         n <= 32768 && k <= 32768;
}

uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

}  // namespace

extern "C" {

int bgc_diag_abi_version(void) { return BGC_DIAG_ABI_VERSION; }

const char* bgc_diag_last_error(void) { return g_last_error.c_str(); }

int bgc_diag_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int bgc_diag_device_arch(int device, char* buf, size_t len) {
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  std::snprintf(buf, len, "%s", prop.gcnArchName);
  return 0;
}

int bgc_diag_hbm(int device, uint64_t bytes, int iters, uint32_t seed, bgc_hbm_result* out) {
  if (!out || iters <= 0 || bytes < (1u << 20)) {
    g_last_error = "invalid arguments";
    return 1;
  }
  std::memset(out, 0, sizeof(*out));
  bytes &= ~static_cast<uint64_t>(15);
  const uint64_t n16 = bytes / 16;
  HIP_TRY(hipSetDevice(device));
  DeviceBuffer a, b, counters;
  HIP_TRY(hipMalloc(&a.p, bytes));
  HIP_TRY(hipMalloc(&b.p, bytes));
  HIP_TRY(hipMalloc(&counters.p, 2 * sizeof(unsigned long long)));
  auto* bad = static_cast<unsigned long long*>(counters.p);
  unsigned long long init[2] = {0ULL, ~0ULL};
  HIP_TRY(hipMemcpy(bad, init, sizeof(init), hipMemcpyHostToDevice));
  const int grid = cu_count(device) * 8;
  Events ev;
  HIP_TRY(hipEventCreate(&ev.a));
  HIP_TRY(hipEventCreate(&ev.b));
  auto t0 = hipEventRecord(ev.a, nullptr);
  (void)t0;
  float best_fill = 1e30f, best_copy = 1e30f, best_check = 1e30f, ms = 0.f;
  float total = 0.f;
  // warm-up (also first-touch of the pages)
  hipLaunchKernelGGL(hbm_fill, dim3(grid), dim3(kBlock), 0, nullptr, static_cast<u32x4*>(a.p), n16, seed);
  HIP_TRY(hipGetLastError());
  for (int it = 0; it < iters; ++it) {
    HIP_TRY(hipEventRecord(ev.a, nullptr));
    hipLaunchKernelGGL(hbm_fill, dim3(grid), dim3(kBlock), 0, nullptr, static_cast<u32x4*>(a.p), n16, seed);
    HIP_TRY(hipEventRecord(ev.b, nullptr));
    HIP_TRY(hipEventSynchronize(ev.b));
    HIP_TRY(hipEventElapsedTime(&ms, ev.a, ev.b));
    best_fill = std::min(best_fill, ms);
    total += ms;
    HIP_TRY(hipEventRecord(ev.a, nullptr));
    hipLaunchKernelGGL(hbm_copy, dim3(grid), dim3(kBlock), 0, nullptr, static_cast<const u32x4*>(a.p),
                       static_cast<u32x4*>(b.p), n16);
    HIP_TRY(hipEventRecord(ev.b, nullptr));
    HIP_TRY(hipEventSynchronize(ev.b));
    HIP_TRY(hipEventElapsedTime(&ms, ev.a, ev.b));
    best_copy = std::min(best_copy, ms);
    total += ms;
    HIP_TRY(hipEventRecord(ev.a, nullptr));
    hipLaunchKernelGGL(hbm_check, dim3(grid), dim3(kBlock), 0, nullptr, static_cast<const u32x4*>(b.p), n16, seed,
                       bad, bad + 1);
    HIP_TRY(hipEventRecord(ev.b, nullptr));
    HIP_TRY(hipEventSynchronize(ev.b));
    HIP_TRY(hipEventElapsedTime(&ms, ev.a, ev.b));
    best_check = std::min(best_check, ms);
    total += ms;
  }
  HIP_TRY(hipGetLastError());
  unsigned long long res[2];
  HIP_TRY(hipMemcpy(res, bad, sizeof(res), hipMemcpyDeviceToHost));
  out->bytes = bytes;
  out->iters = iters;
  out->write_gbps = static_cast<double>(bytes) / (best_fill * 1e-3) / 1e9;
  out->copy_gbps = 2.0 * static_cast<double>(bytes) / (best_copy * 1e-3) / 1e9;
  out->read_gbps = static_cast<double>(bytes) / (best_check * 1e-3) / 1e9;
  out->mismatches = res[0];
  out->first_bad_word = res[1];
  out->elapsed_ms = total;
  return 0;
}

int bgc_diag_mfma(int device, int waves_per_cu, int throughput_iters, uint32_t seed, bgc_mfma_result* out) {
  if (!out || waves_per_cu <= 0 || throughput_iters <= 0 || throughput_iters > (1 << 18)) {
    g_last_error = "invalid arguments";
    return 1;
  }
  std::memset(out, 0, sizeof(*out));
  HIP_TRY(hipSetDevice(device));
  const int cus = cu_count(device);
  const int blocks = std::max(1, cus * waves_per_cu / (kBlock / 64));
  const int rounds = 8;
  DeviceBuffer tiles, bad, fails, xticks, xwaves;
  HIP_TRY(hipMalloc(&tiles.p, BGC_DIAG_MAX_CU_KEYS * sizeof(unsigned)));
  HIP_TRY(hipMalloc(&bad.p, BGC_DIAG_MAX_CU_KEYS * sizeof(unsigned)));
  HIP_TRY(hipMalloc(&fails.p, sizeof(unsigned)));
  HIP_TRY(hipMalloc(&xticks.p, 8 * sizeof(unsigned long long)));
  HIP_TRY(hipMalloc(&xwaves.p, 8 * sizeof(unsigned)));
  HIP_TRY(hipMemset(tiles.p, 0, BGC_DIAG_MAX_CU_KEYS * sizeof(unsigned)));
  HIP_TRY(hipMemset(bad.p, 0, BGC_DIAG_MAX_CU_KEYS * sizeof(unsigned)));
  HIP_TRY(hipMemset(fails.p, 0, sizeof(unsigned)));
  Events ev;
  HIP_TRY(hipEventCreate(&ev.a));
  HIP_TRY(hipEventCreate(&ev.b));
  float ms_check = 0.f, ms_tp = 0.f;
  HIP_TRY(hipEventRecord(ev.a, nullptr));
  hipLaunchKernelGGL(mfma_check, dim3(blocks), dim3(kBlock), 0, nullptr, seed, rounds,
                     static_cast<unsigned*>(tiles.p), static_cast<unsigned*>(bad.p));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(ev.b, nullptr));
  HIP_TRY(hipEventSynchronize(ev.b));
  HIP_TRY(hipEventElapsedTime(&ms_check, ev.a, ev.b));
  // warm-up then timed throughput pass
  auto* xt = static_cast<unsigned long long*>(xticks.p);
  auto* xw = static_cast<unsigned*>(xwaves.p);
  hipLaunchKernelGGL(mfma_throughput, dim3(blocks), dim3(kBlock), 0, nullptr, seed, 64, static_cast<unsigned*>(fails.p),
                     xt, xw);
  HIP_TRY(hipMemset(fails.p, 0, sizeof(unsigned)));
  HIP_TRY(hipMemset(xticks.p, 0, 8 * sizeof(unsigned long long)));
  HIP_TRY(hipMemset(xwaves.p, 0, 8 * sizeof(unsigned)));
  HIP_TRY(hipEventRecord(ev.a, nullptr));
  hipLaunchKernelGGL(mfma_throughput, dim3(blocks), dim3(kBlock), 0, nullptr, seed, throughput_iters,
                     static_cast<unsigned*>(fails.p), xt, xw);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(ev.b, nullptr));
  HIP_TRY(hipEventSynchronize(ev.b));
  HIP_TRY(hipEventElapsedTime(&ms_tp, ev.a, ev.b));
  std::vector<unsigned> h_tiles(BGC_DIAG_MAX_CU_KEYS), h_bad(BGC_DIAG_MAX_CU_KEYS);
  unsigned h_fails = 0;
  HIP_TRY(hipMemcpy(h_tiles.data(), tiles.p, h_tiles.size() * sizeof(unsigned), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(h_bad.data(), bad.p, h_bad.size() * sizeof(unsigned), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&h_fails, fails.p, sizeof(unsigned), hipMemcpyDeviceToHost));
  unsigned long long h_ticks[8];
  unsigned h_waves[8];
  HIP_TRY(hipMemcpy(h_ticks, xticks.p, sizeof(h_ticks), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(h_waves, xwaves.p, sizeof(h_waves), hipMemcpyDeviceToHost));
  int rate_khz = 0;
  if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || rate_khz <= 0) {
    rate_khz = 100000;  // CDNA constant clock: 100 MHz
  }
  double lo = 0, hi = 0;
  for (int x = 0; x < 8; ++x) {
    out->xcc_waves[x] = static_cast<int>(h_waves[x]);
    out->xcc_wave_us[x] = h_waves[x] ? static_cast<double>(h_ticks[x]) / h_waves[x] / (rate_khz * 1e-3) : 0.0;
    if (!h_waves[x]) continue;
    lo = lo == 0 ? out->xcc_wave_us[x] : std::min(lo, out->xcc_wave_us[x]);
    hi = std::max(hi, out->xcc_wave_us[x]);
  }
  out->xcc_balance = hi > 0 ? lo / hi : 0.0;
  bool xcc_seen[8] = {false};
  for (int k = 0; k < BGC_DIAG_MAX_CU_KEYS; ++k) {
    if (!h_tiles[static_cast<size_t>(k)]) continue;
    out->cus_seen++;
    out->tiles_checked += h_tiles[static_cast<size_t>(k)];
    xcc_seen[(k >> 8) & 7] = true;
    if (h_bad[static_cast<size_t>(k)]) {
      out->mismatches += h_bad[static_cast<size_t>(k)];
      if (out->bad_cus < 64) out->bad_cu_keys[out->bad_cus] = k;
      out->bad_cus++;
    }
  }
  for (bool s : xcc_seen) out->xccs_seen += s ? 1 : 0;
  const double waves = static_cast<double>(blocks) * (kBlock / 64);
  const double flops = waves * throughput_iters * 4.0 * (2.0 * 16 * 16 * 32);
  out->tflops = flops / (ms_tp * 1e-3) / 1e12;
  out->throughput_ok = h_fails == 0;
  out->elapsed_ms = ms_check + ms_tp;
  return 0;
}

int bgc_diag_mfma_lowp(int device, int waves_per_cu, int throughput_iters, uint32_t seed, bgc_lowp_result* out) {
  if (!out || waves_per_cu <= 0 || waves_per_cu > 64 || throughput_iters <= 0 || throughput_iters > (1 << 16)) {
    g_last_error = "invalid arguments";
    return 1;
  }
  std::memset(out, 0, sizeof(*out));
  HIP_TRY(hipSetDevice(device));
  const int cus = cu_count(device);
  const int blocks = std::max(1, cus * waves_per_cu / (kBlock / 64));
  const int rounds = 2;
  // bins: [fmt][scaled] tiles and mismatches per CU key
  DeviceBuffer tiles, bad, fails;
  const size_t bins = 4 * static_cast<size_t>(BGC_DIAG_MAX_CU_KEYS);
  HIP_TRY(hipMalloc(&tiles.p, bins * sizeof(unsigned)));
  HIP_TRY(hipMalloc(&bad.p, bins * sizeof(unsigned)));
  HIP_TRY(hipMalloc(&fails.p, 2 * sizeof(unsigned)));
  HIP_TRY(hipMemset(tiles.p, 0, bins * sizeof(unsigned)));
  HIP_TRY(hipMemset(bad.p, 0, bins * sizeof(unsigned)));
  auto* t = static_cast<unsigned*>(tiles.p);
  auto* b = static_cast<unsigned*>(bad.p);
  auto* f = static_cast<unsigned*>(fails.p);
  Events ev;
  HIP_TRY(hipEventCreate(&ev.a));
  HIP_TRY(hipEventCreate(&ev.b));
  float ms = 0.f, total = 0.f;
  HIP_TRY(hipEventRecord(ev.a, nullptr));
  for (int sc = 0; sc < 2; ++sc) {
    const size_t o8 = static_cast<size_t>(sc) * BGC_DIAG_MAX_CU_KEYS, o4 = (2 + static_cast<size_t>(sc)) * BGC_DIAG_MAX_CU_KEYS;
    hipLaunchKernelGGL(mfma_lowp_check<0>, dim3(blocks), dim3(kBlock), 0, nullptr, seed, rounds, sc, t + o8, b + o8);
    hipLaunchKernelGGL(mfma_lowp_check<4>, dim3(blocks), dim3(kBlock), 0, nullptr, seed, rounds, sc, t + o4, b + o4);
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(ev.b, nullptr));
  HIP_TRY(hipEventSynchronize(ev.b));
  HIP_TRY(hipEventElapsedTime(&ms, ev.a, ev.b));
  total += ms;
  // warm-up, then one timed launch per format
  hipLaunchKernelGGL(mfma_lowp_throughput<0>, dim3(blocks), dim3(kBlock), 0, nullptr, seed, 64, f);
  HIP_TRY(hipMemset(f, 0, 2 * sizeof(unsigned)));
  float ms_fmt[2] = {0.f, 0.f};
  for (int i = 0; i < 2; ++i) {
    HIP_TRY(hipEventRecord(ev.a, nullptr));
    if (i == 0) {
      hipLaunchKernelGGL(mfma_lowp_throughput<0>, dim3(blocks), dim3(kBlock), 0, nullptr, seed, throughput_iters, f);
    } else {
      hipLaunchKernelGGL(mfma_lowp_throughput<4>, dim3(blocks), dim3(kBlock), 0, nullptr, seed, throughput_iters, f + 1);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ev.b, nullptr));
    HIP_TRY(hipEventSynchronize(ev.b));
    HIP_TRY(hipEventElapsedTime(&ms_fmt[i], ev.a, ev.b));
    total += ms_fmt[i];
  }
  std::vector<unsigned> h_t(bins), h_b(bins);
  unsigned h_f[2] = {0, 0};
  HIP_TRY(hipMemcpy(h_t.data(), t, bins * sizeof(unsigned), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(h_b.data(), b, bins * sizeof(unsigned), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(h_f, f, sizeof(h_f), hipMemcpyDeviceToHost));
  uint64_t* mism[4] = {&out->fp8_mismatches, &out->fp8_scaled_mismatches, &out->fp4_mismatches,
                       &out->fp4_scaled_mismatches};
  for (int k = 0; k < BGC_DIAG_MAX_CU_KEYS; ++k) {
    unsigned seen = 0, bad_here = 0;
    for (int v = 0; v < 4; ++v) {
      const size_t i = static_cast<size_t>(v) * BGC_DIAG_MAX_CU_KEYS + static_cast<size_t>(k);
      seen += h_t[i];
      bad_here += h_b[i];
      *mism[v] += h_b[i];
      out->tiles_checked += h_t[i];
    }
    if (!seen) continue;
    out->cus_seen++;
    if (bad_here) {
      if (out->bad_cus < 64) out->bad_cu_keys[out->bad_cus] = k;
      out->bad_cus++;
    }
  }
  const double waves = static_cast<double>(blocks) * (kBlock / 64);
  const double flops = waves * throughput_iters * 4.0 * (2.0 * 16 * 16 * 128);
  out->fp8_tflops = ms_fmt[0] > 0 ? flops / (ms_fmt[0] * 1e-3) / 1e12 : 0.0;
  out->fp4_tflops = ms_fmt[1] > 0 ? flops / (ms_fmt[1] * 1e-3) / 1e12 : 0.0;
  out->throughput_ok = h_f[0] == 0 && h_f[1] == 0;
  out->elapsed_ms = total;
  return 0;
}

int bgc_diag_burn(int device, int duration_ms, int waves_per_cu, uint32_t seed, bgc_burn_result* out) {
  return bgc_diag_burn_dtype(device, duration_ms, waves_per_cu, seed, BGC_BURN_BF16, out);
}

int bgc_diag_burn_dtype(int device, int duration_ms, int waves_per_cu, uint32_t seed, int dtype, bgc_burn_result* out) {
  if (!out || duration_ms <= 0 || duration_ms > 600000 || waves_per_cu <= 0 || waves_per_cu > 64 ||
      dtype < BGC_BURN_BF16 || dtype > BGC_BURN_FP4) {
    g_last_error = "invalid arguments";
    return 1;
  }
  std::memset(out, 0, sizeof(*out));
  HIP_TRY(hipSetDevice(device));
  const int cus = cu_count(device);
  const int blocks = std::max(1, cus * waves_per_cu / (kBlock / 64));
  DeviceBuffer fails, xticks, xwaves;
  HIP_TRY(hipMalloc(&fails.p, sizeof(unsigned)));
  HIP_TRY(hipMalloc(&xticks.p, 8 * sizeof(unsigned long long)));
  HIP_TRY(hipMalloc(&xwaves.p, 8 * sizeof(unsigned)));
  HIP_TRY(hipMemset(fails.p, 0, sizeof(unsigned)));
  auto* xt = static_cast<unsigned long long*>(xticks.p);
  auto* xw = static_cast<unsigned*>(xwaves.p);
  Events ev, total;
  HIP_TRY(hipEventCreate(&ev.a));
  HIP_TRY(hipEventCreate(&ev.b));
  HIP_TRY(hipEventCreate(&total.a));
  HIP_TRY(hipEventCreate(&total.b));
  // size one launch to ~10 ms at MI355X rates (iters * 4 MFMA per wave), measured below
  int iters = 2048;
  const double mfma_k = dtype == BGC_BURN_BF16 ? 32.0 : 128.0;  // 16x16x32 bf16, 16x16x128 MX
  const double flops_per_iter = static_cast<double>(blocks) * (kBlock / 64) * 4.0 * (2.0 * 16 * 16 * mfma_k);
  auto* fp = static_cast<unsigned*>(fails.p);
  float ms = 0.f;
  HIP_TRY(hipEventRecord(total.a, nullptr));
  double sum_flops = 0;
  while (true) {
    HIP_TRY(hipEventRecord(ev.a, nullptr));
    if (dtype == BGC_BURN_FP8) {
      hipLaunchKernelGGL(mfma_lowp_throughput<0>, dim3(blocks), dim3(kBlock), 0, nullptr, seed, iters, fp);
    } else if (dtype == BGC_BURN_FP4) {
      hipLaunchKernelGGL(mfma_lowp_throughput<4>, dim3(blocks), dim3(kBlock), 0, nullptr, seed, iters, fp);
    } else {
      hipLaunchKernelGGL(mfma_throughput, dim3(blocks), dim3(kBlock), 0, nullptr, seed, iters, fp, xt, xw);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ev.b, nullptr));
    HIP_TRY(hipEventSynchronize(ev.b));
    HIP_TRY(hipEventElapsedTime(&ms, ev.a, ev.b));
    const double tf = flops_per_iter * iters / (ms * 1e-3) / 1e12;
    out->tflops_max = std::max(out->tflops_max, tf);
    if (out->launches == 0) {
      out->tflops_first = tf;
      out->tflops_min = tf;
      // retune the launch length to ~10 ms now that the rate is known
      iters = std::max(64, std::min(1 << 18, static_cast<int>(iters * (10.0 / std::max(0.01f, ms)))));
    } else {
      out->tflops_min = std::min(out->tflops_min, tf);
    }
    out->tflops_last = tf;
    out->launches++;
    sum_flops += flops_per_iter * (out->launches == 1 ? 2048 : iters);
    HIP_TRY(hipEventRecord(total.b, nullptr));
    HIP_TRY(hipEventSynchronize(total.b));
    float so_far = 0.f;
    HIP_TRY(hipEventElapsedTime(&so_far, total.a, total.b));
    out->elapsed_ms = so_far;
    if (so_far >= static_cast<float>(duration_ms)) break;
  }
  unsigned h_fails = 0;
  HIP_TRY(hipMemcpy(&h_fails, fails.p, sizeof(unsigned), hipMemcpyDeviceToHost));
  out->mismatches = h_fails;
  out->tflops_mean = sum_flops / (out->elapsed_ms * 1e-3) / 1e12;
  return 0;
}

int bgc_diag_gemm(int device, int m, int n, int k, const uint16_t* a_bf16, const uint16_t* b_bf16, float* c) {
  if (!a_bf16 || !b_bf16 || !c || m <= 0 || n <= 0 || k <= 0 || m % 16 || n % 16 || k % 32 || m > 4096 ||
      n > 4096 || k > 8192) {
    g_last_error = "invalid arguments (M, N multiples of 16 up to 4096; K a multiple of 32 up to 8192)";
    return 1;
  }
  HIP_TRY(hipSetDevice(device));
  const size_t a_bytes = static_cast<size_t>(m) * k * 2, b_bytes = static_cast<size_t>(k) * n * 2;
  const size_t c_bytes = static_cast<size_t>(m) * n * 4;
  DeviceBuffer da, db, dc;
  HIP_TRY(hipMalloc(&da.p, a_bytes));
  HIP_TRY(hipMalloc(&db.p, b_bytes));
  HIP_TRY(hipMalloc(&dc.p, c_bytes));
  HIP_TRY(hipMemcpy(da.p, a_bf16, a_bytes, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(db.p, b_bf16, b_bytes, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(mfma_gemm, dim3(n / 16, m / 16), dim3(64), 0, nullptr, static_cast<const __bf16*>(da.p),
                     static_cast<const __bf16*>(db.p), static_cast<float*>(dc.p), m, n, k);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpy(c, dc.p, c_bytes, hipMemcpyDeviceToHost));
  return 0;
}

int bgc_diag_pcie(int device, uint64_t bytes, int iters, uint32_t seed, bgc_pcie_result* out) {
  if (!out || iters <= 0 || bytes < (1u << 20) || bytes > (uint64_t{16} << 30)) {
    g_last_error = "invalid arguments";
    return 1;
  }
  std::memset(out, 0, sizeof(*out));
  bytes &= ~static_cast<uint64_t>(7);
  const uint64_t words = bytes / 8;
  HIP_TRY(hipSetDevice(device));
  HostBuffer src, dst, src2;
  DeviceBuffer d1, d2;
  HIP_TRY(hipHostMalloc(&src.p, bytes, hipHostMallocDefault));
  HIP_TRY(hipHostMalloc(&dst.p, bytes, hipHostMallocDefault));
  HIP_TRY(hipHostMalloc(&src2.p, bytes, hipHostMallocDefault));
  HIP_TRY(hipMalloc(&d1.p, bytes));
  HIP_TRY(hipMalloc(&d2.p, bytes));
  auto* s64 = static_cast<uint64_t*>(src.p);
  for (uint64_t i = 0; i < words; ++i) s64[i] = (static_cast<uint64_t>(mix32(static_cast<uint32_t>(i) ^ seed)) << 32) | mix32(static_cast<uint32_t>(i >> 32) + seed + 1);
  std::memset(dst.p, 0, bytes);
  std::memset(src2.p, 0x5a, bytes);
  Streams st;
  HIP_TRY(hipStreamCreateWithFlags(&st.a, hipStreamNonBlocking));
  HIP_TRY(hipStreamCreateWithFlags(&st.b, hipStreamNonBlocking));
  Events ev, ev2;
  HIP_TRY(hipEventCreate(&ev.a));
  HIP_TRY(hipEventCreate(&ev.b));
  HIP_TRY(hipEventCreate(&ev2.a));
  HIP_TRY(hipEventCreate(&ev2.b));
  // warm-up both directions (page tables, DMA engine clocks)
  HIP_TRY(hipMemcpyAsync(d1.p, src.p, bytes, hipMemcpyHostToDevice, st.a));
  HIP_TRY(hipMemcpyAsync(d2.p, d1.p, bytes, hipMemcpyDeviceToDevice, st.a));
  HIP_TRY(hipMemcpyAsync(dst.p, d2.p, bytes, hipMemcpyDeviceToHost, st.a));
  HIP_TRY(hipStreamSynchronize(st.a));
  // round trip check: the pattern went host -> device -> device -> host
  const auto* d64 = static_cast<const uint64_t*>(dst.p);
  uint64_t bad = 0;
  for (uint64_t i = 0; i < words; ++i) bad += d64[i] != s64[i];
  float best_h2d = 1e30f, best_d2h = 1e30f, ms = 0.f, total = 0.f;
  double best_bidir = 0;
  for (int it = 0; it < iters; ++it) {
    HIP_TRY(hipEventRecord(ev.a, st.a));
    HIP_TRY(hipMemcpyAsync(d1.p, src.p, bytes, hipMemcpyHostToDevice, st.a));
    HIP_TRY(hipEventRecord(ev.b, st.a));
    HIP_TRY(hipEventSynchronize(ev.b));
    HIP_TRY(hipEventElapsedTime(&ms, ev.a, ev.b));
    best_h2d = std::min(best_h2d, ms);
    total += ms;
    HIP_TRY(hipEventRecord(ev.a, st.a));
    HIP_TRY(hipMemcpyAsync(dst.p, d1.p, bytes, hipMemcpyDeviceToHost, st.a));
    HIP_TRY(hipEventRecord(ev.b, st.a));
    HIP_TRY(hipEventSynchronize(ev.b));
    HIP_TRY(hipEventElapsedTime(&ms, ev.a, ev.b));
    best_d2h = std::min(best_d2h, ms);
    total += ms;
    // both directions at once: H2D on one stream, D2H on the other
    HIP_TRY(hipEventRecord(ev.a, st.a));
    HIP_TRY(hipEventRecord(ev2.a, st.b));
    HIP_TRY(hipMemcpyAsync(d2.p, src2.p, bytes, hipMemcpyHostToDevice, st.a));
    HIP_TRY(hipMemcpyAsync(dst.p, d1.p, bytes, hipMemcpyDeviceToHost, st.b));
    HIP_TRY(hipEventRecord(ev.b, st.a));
    HIP_TRY(hipEventRecord(ev2.b, st.b));
    HIP_TRY(hipEventSynchronize(ev.b));
    HIP_TRY(hipEventSynchronize(ev2.b));
    float ms_a = 0.f, ms_b = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms_a, ev.a, ev.b));
    HIP_TRY(hipEventElapsedTime(&ms_b, ev2.a, ev2.b));
    const double span = std::max(ms_a, ms_b);
    best_bidir = std::max(best_bidir, 2.0 * static_cast<double>(bytes) / (span * 1e-3) / 1e9);
    total += static_cast<float>(span);
  }
  HIP_TRY(hipGetLastError());
  out->bytes = bytes;
  out->iters = iters;
  out->h2d_gbps = static_cast<double>(bytes) / (best_h2d * 1e-3) / 1e9;
  out->d2h_gbps = static_cast<double>(bytes) / (best_d2h * 1e-3) / 1e9;
  out->bidir_gbps = best_bidir;
  out->mismatches = bad;
  out->elapsed_ms = total;
  return 0;
}

int bgc_diag_gemm_soak(int device, int m, int n, int k, int launches, uint32_t seed, bgc_soak_result* out) {
  if (!out || launches <= 0 || !soak_shape_ok(m, n, k)) {
    g_last_error = "invalid arguments: m, n multiples of 128 and k of 64 (each <= 32768)";
    return 1;
  }
  const bool big = soak_big_tile(m, n);
  std::memset(out, 0, sizeof(*out));
  HIP_TRY(hipSetDevice(device));
  const size_t na = static_cast<size_t>(m) * k, nb = static_cast<size_t>(n) * k, nc = static_cast<size_t>(m) * n;
  DeviceBuffer a, bt, c, sa, sb, rref, cref, rgot, cgot;
  HIP_TRY(hipMalloc(&a.p, na * 2));
  HIP_TRY(hipMalloc(&bt.p, nb * 2));
  HIP_TRY(hipMalloc(&c.p, nc * 4));
  HIP_TRY(hipMalloc(&sa.p, static_cast<size_t>(k) * 4));
  HIP_TRY(hipMalloc(&sb.p, static_cast<size_t>(k) * 4));
  HIP_TRY(hipMalloc(&rref.p, static_cast<size_t>(m) * 8));
  HIP_TRY(hipMalloc(&cref.p, static_cast<size_t>(n) * 8));
  HIP_TRY(hipMalloc(&rgot.p, static_cast<size_t>(m) * 8));
  HIP_TRY(hipMalloc(&cgot.p, static_cast<size_t>(n) * 8));
  const int fill_grid = cu_count(device) * 8;
  hipLaunchKernelGGL(soak_fill, dim3(fill_grid), dim3(kBlock), 0, nullptr, static_cast<__bf16*>(a.p), na, seed);
  hipLaunchKernelGGL(soak_fill, dim3(fill_grid), dim3(kBlock), 0, nullptr, static_cast<__bf16*>(bt.p), nb, seed ^ 0xB7B7B7B7u);
  HIP_TRY(hipGetLastError());
  // reference checksums on an integer path: sA = 1^T A (per k), sB = B 1 = per-k sums of Bt's rows
  HIP_TRY(hipMemset(sa.p, 0, static_cast<size_t>(k) * 4));
  HIP_TRY(hipMemset(sb.p, 0, static_cast<size_t>(k) * 4));
  hipLaunchKernelGGL(soak_colsum, dim3((k + kBlock - 1) / kBlock, (m + 63) / 64), dim3(kBlock), 0, nullptr,
                     static_cast<const __bf16*>(a.p), m, k, static_cast<int*>(sa.p));
  hipLaunchKernelGGL(soak_colsum, dim3((k + kBlock - 1) / kBlock, (n + 63) / 64), dim3(kBlock), 0, nullptr,
                     static_cast<const __bf16*>(bt.p), n, k, static_cast<int*>(sb.p));
  hipLaunchKernelGGL(soak_rowdot, dim3(m), dim3(kBlock), 0, nullptr, static_cast<const __bf16*>(a.p), k,
                     static_cast<const int*>(sb.p), static_cast<long long*>(rref.p));  // rows of C = A (B 1)
  hipLaunchKernelGGL(soak_rowdot, dim3(n), dim3(kBlock), 0, nullptr, static_cast<const __bf16*>(bt.p), k,
                     static_cast<const int*>(sa.p), static_cast<long long*>(cref.p));  // cols of C = (1^T A) B
  HIP_TRY(hipGetLastError());
  std::vector<long long> rr(static_cast<size_t>(m)), cr(static_cast<size_t>(n)), rg(static_cast<size_t>(m)),
      cg(static_cast<size_t>(n));
  HIP_TRY(hipMemcpy(rr.data(), rref.p, rr.size() * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(cr.data(), cref.p, cr.size() * 8, hipMemcpyDeviceToHost));
  auto verify = [&](uint64_t* row_bad, uint64_t* col_bad) -> int {
    HIP_TRY(hipMemset(cgot.p, 0, static_cast<size_t>(n) * 8));
    hipLaunchKernelGGL(soak_c_rowsum, dim3(m), dim3(kBlock), 0, nullptr, static_cast<const float*>(c.p), n,
                       static_cast<long long*>(rgot.p));
    hipLaunchKernelGGL(soak_c_colsum, dim3((n + kBlock - 1) / kBlock, (m + 63) / 64), dim3(kBlock), 0, nullptr,
                       static_cast<const float*>(c.p), m, n, static_cast<unsigned long long*>(cgot.p));
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy(rg.data(), rgot.p, rg.size() * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(cg.data(), cgot.p, cg.size() * 8, hipMemcpyDeviceToHost));
    for (int i = 0; i < m; ++i) *row_bad += rg[static_cast<size_t>(i)] != rr[static_cast<size_t>(i)];
    for (int j = 0; j < n; ++j) *col_bad += cg[static_cast<size_t>(j)] != cr[static_cast<size_t>(j)];
    return 0;
  };
  Events ev;
  HIP_TRY(hipEventCreate(&ev.a));
  HIP_TRY(hipEventCreate(&ev.b));
  const double flop = 2.0 * m * n * static_cast<double>(k);
  float ms = 0.f, best = 1e30f, total = 0.f;
  for (int it = 0; it < launches; ++it) {
    // poison C before the last checked launch, so its checksums cover that launch's writes
    if (it > 0 && it == launches - 1) HIP_TRY(hipMemsetAsync(c.p, 0xFF, nc * 4, nullptr));
    HIP_TRY(hipEventRecord(ev.a, nullptr));
    launch_soak_gemm(big, a.p, bt.p, c.p, m, n, k, nullptr);
    HIP_TRY(hipEventRecord(ev.b, nullptr));
    HIP_TRY(hipEventSynchronize(ev.b));
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventElapsedTime(&ms, ev.a, ev.b));
    best = std::min(best, ms);
    total += ms;
    if (it == 0 && verify(&out->row_mismatches, &out->col_mismatches) != 0) return 1;
  }
  if (launches > 1 && verify(&out->row_mismatches, &out->col_mismatches) != 0) return 1;
  out->m = m;
  out->n = n;
  out->k = k;
  out->tile = big ? 256 : 128;
  out->kernel = soak_pingpong(big, k) ? 2 : 1;
  out->launches = launches;
  out->elapsed_ms = total;
  out->tflops_best = flop / (best * 1e-3) / 1e12;
  out->tflops_mean = flop * launches / (total * 1e-3) / 1e12;
  return 0;
}

int bgc_diag_gemm_tiled(int device, int m, int n, int k, const uint16_t* a_bf16, const uint16_t* bt_bf16, float* c) {
  if (!a_bf16 || !bt_bf16 || !c || !soak_shape_ok(m, n, k)) {
    g_last_error = "invalid arguments: m, n multiples of 128 and k of 64 (each <= 32768)";
    return 1;
  }
  HIP_TRY(hipSetDevice(device));
  const size_t na = static_cast<size_t>(m) * k, nb = static_cast<size_t>(n) * k, nc = static_cast<size_t>(m) * n;
  DeviceBuffer da, db, dc;
  HIP_TRY(hipMalloc(&da.p, na * 2));
  HIP_TRY(hipMalloc(&db.p, nb * 2));
  HIP_TRY(hipMalloc(&dc.p, nc * 4));
  HIP_TRY(hipMemcpy(da.p, a_bf16, na * 2, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(db.p, bt_bf16, nb * 2, hipMemcpyHostToDevice));
  HIP_TRY(hipMemset(dc.p, 0xFF, nc * 4));  // NaN: an element the kernel never writes cannot pass
  launch_soak_gemm(soak_big_tile(m, n), da.p, db.p, dc.p, m, n, k, nullptr);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpy(c, dc.p, nc * 4, hipMemcpyDeviceToHost));
  return 0;
}

int bgc_diag_mx_gemm(int device, int fmt, int m, int n, int k, const uint8_t* a, const uint8_t* a_scales,
                     const uint8_t* bt, const uint8_t* bt_scales, float* c) {
  if (!a || !a_scales || !bt || !bt_scales || !c || (fmt != 0 && fmt != 4) || m <= 0 || n <= 0 || k <= 0 ||
      m % 16 || n % 16 || k % 128 || m > 16384 || n > 16384 || k > 65536) {
    g_last_error = "invalid arguments: fmt 0 (fp8 e4m3) or 4 (fp4 e2m1); m, n multiples of 16 (<= 16384), k of 128 (<= 65536)";
    return 1;
  }
  HIP_TRY(hipSetDevice(device));
  const size_t code_bytes_a = fmt == 0 ? static_cast<size_t>(m) * k : static_cast<size_t>(m) * k / 2;
  const size_t code_bytes_b = fmt == 0 ? static_cast<size_t>(n) * k : static_cast<size_t>(n) * k / 2;
  const size_t sa_bytes = static_cast<size_t>(m) * (k / 32), sb_bytes = static_cast<size_t>(n) * (k / 32);
  const size_t nc = static_cast<size_t>(m) * n;
  DeviceBuffer da, dsa, db, dsb, dc;
  HIP_TRY(hipMalloc(&da.p, code_bytes_a));
  HIP_TRY(hipMalloc(&dsa.p, sa_bytes));
  HIP_TRY(hipMalloc(&db.p, code_bytes_b));
  HIP_TRY(hipMalloc(&dsb.p, sb_bytes));
  HIP_TRY(hipMalloc(&dc.p, nc * 4));
  HIP_TRY(hipMemcpy(da.p, a, code_bytes_a, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(dsa.p, a_scales, sa_bytes, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(db.p, bt, code_bytes_b, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(dsb.p, bt_scales, sb_bytes, hipMemcpyHostToDevice));
  HIP_TRY(hipMemset(dc.p, 0xFF, nc * 4));  // NaN: an element the kernel never writes cannot pass
  const dim3 grid(static_cast<unsigned>((m / 16) * (n / 16)));
  const auto* pa = static_cast<const uint8_t*>(da.p);
  const auto* psa = static_cast<const uint8_t*>(dsa.p);
  const auto* pb = static_cast<const uint8_t*>(db.p);
  const auto* psb = static_cast<const uint8_t*>(dsb.p);
  if (fmt == 0) {
    hipLaunchKernelGGL(mx_gemm<0>, grid, dim3(64), 0, nullptr, pa, psa, pb, psb, static_cast<float*>(dc.p), m, n, k);
  } else {
    hipLaunchKernelGGL(mx_gemm<4>, grid, dim3(64), 0, nullptr, pa, psa, pb, psb, static_cast<float*>(dc.p), m, n, k);
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpy(c, dc.p, nc * 4, hipMemcpyDeviceToHost));
  return 0;
}

int bgc_diag_hbm_walk(int device, double fraction, uint64_t chunk_bytes, int budget_ms, uint32_t seed,
                      bgc_hbm_walk_result* out) {
  constexpr uint64_t kMinChunk = 64ULL << 20;
  if (!out || !(fraction > 0.0 && fraction <= 0.99) || chunk_bytes < kMinChunk || budget_ms <= 0) {
    g_last_error = "invalid arguments: 0 < fraction <= 0.99, chunk_bytes >= 64 MiB, budget_ms > 0";
    return 1;
  }
  std::memset(out, 0, sizeof(*out));
  const auto t0 = std::chrono::steady_clock::now();
  auto elapsed_ms = [&] {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  };
  HIP_TRY(hipSetDevice(device));
  DeviceBuffer counters;  // before the walk takes the memory
  HIP_TRY(hipMalloc(&counters.p, 2 * sizeof(unsigned long long)));
  size_t free_b = 0, total_b = 0;
  HIP_TRY(hipMemGetInfo(&free_b, &total_b));
  out->free_bytes = free_b;
  out->total_bytes = total_b;
  const uint64_t align = 2ULL << 20;
  const uint64_t target = static_cast<uint64_t>(fraction * static_cast<double>(free_b)) & ~(align - 1);
  out->target_bytes = target;
  Chunks chunks;
  uint64_t got = 0, cb = chunk_bytes & ~(align - 1);
  while (got < target) {
    const uint64_t want = std::min(cb, target - got);
    void* p = nullptr;
    if (hipMalloc(&p, want) != hipSuccess || !p) {
      (void)hipGetLastError();  // clear the sticky allocation error
      if (cb <= kMinChunk) break;
      cb = std::max(kMinChunk, (cb / 2) & ~(align - 1));
      continue;
    }
    chunks.v.emplace_back(p, want);
    got += want;
  }
  if (chunks.v.empty()) {
    g_last_error = "hbm walk: no device memory could be allocated";
    return 1;
  }
  out->chunks = static_cast<int>(chunks.v.size());
  out->alloc_ms = elapsed_ms();
  auto* bad = static_cast<unsigned long long*>(counters.p);
  const int grid = cu_count(device) * 8;
  Events ev;
  HIP_TRY(hipEventCreate(&ev.a));
  HIP_TRY(hipEventCreate(&ev.b));
  const uint64_t key0 = mix64(0x9e3779b97f4a7c15ULL ^ seed);
  double fill_ms = 0, check_ms = 0;
  for (int pass = 0; pass < 2; ++pass) {
    if (pass > 0 && elapsed_ms() > budget_ms) {
      out->budget_hit = 1;
      break;
    }
    const uint64_t key = pass == 0 ? key0 : ~key0;
    const unsigned long long init[2] = {0ULL, ~0ULL};
    HIP_TRY(hipMemcpy(bad, init, sizeof(init), hipMemcpyHostToDevice));
    float ms = 0.f;
    HIP_TRY(hipEventRecord(ev.a, nullptr));
    for (const auto& c : chunks.v) {
      hipLaunchKernelGGL(walk_fill, dim3(grid), dim3(kBlock), 0, nullptr, static_cast<u32x4*>(c.first), c.second / 16, key);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ev.b, nullptr));
    HIP_TRY(hipEventSynchronize(ev.b));
    HIP_TRY(hipEventElapsedTime(&ms, ev.a, ev.b));
    fill_ms += ms;
    HIP_TRY(hipEventRecord(ev.a, nullptr));
    for (const auto& c : chunks.v) {
      hipLaunchKernelGGL(walk_check, dim3(grid), dim3(kBlock), 0, nullptr, static_cast<const u32x4*>(c.first),
                         c.second / 16, key, bad, bad + 1);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ev.b, nullptr));
    HIP_TRY(hipEventSynchronize(ev.b));
    HIP_TRY(hipEventElapsedTime(&ms, ev.a, ev.b));
    check_ms += ms;
    unsigned long long res[2];
    HIP_TRY(hipMemcpy(res, bad, sizeof(res), hipMemcpyDeviceToHost));
    if (res[0] && !out->mismatches) {  // the first failing pass names the first bad word
      out->first_bad_addr = res[1];
      uint64_t found = 0;
      HIP_TRY(hipMemcpy(&found, reinterpret_cast<void*>(static_cast<uintptr_t>(res[1])), 8, hipMemcpyDeviceToHost));
      out->first_bad_xor = found ^ (static_cast<uint64_t>(res[1]) ^ key);
    }
    out->mismatches += res[0];
    out->passes = pass + 1;
  }
  out->bytes_covered = got;
  const double moved = static_cast<double>(got) * out->passes;
  out->write_gbps = fill_ms > 0 ? moved / (fill_ms * 1e-3) / 1e9 : 0.0;
  out->read_gbps = check_ms > 0 ? moved / (check_ms * 1e-3) / 1e9 : 0.0;
  out->elapsed_ms = elapsed_ms();
  return 0;
}

int bgc_diag_device_bdf(int device, char* buf, size_t len) {
  if (!buf || len < 13) {
    g_last_error = "invalid arguments";
    return 1;
  }
  char tmp[64] = {0};
  HIP_TRY(hipDeviceGetPCIBusId(tmp, static_cast<int>(sizeof(tmp)), device));
  for (char* p = tmp; *p; ++p) *p = static_cast<char>(std::tolower(static_cast<unsigned char>(*p)));
  std::snprintf(buf, len, "%s", tmp);
  return 0;
}

}  // extern "C"
