// C ABI of the MI355X (gfx950) health-diagnostic kernels (libbgc_gpu_diag.so).
//
// The reference has no GPU code; these kernels implement the north
// star's "GPU discovery, health" for the node agent: before a GPU is advertised as
// schedulable `amd.com/gpu`, its HBM3E is pattern-tested at streaming bandwidth and
// every CU's matrix cores are checked with exact-integer MFMA tiles.  The library is
// dlopen()ed by the node agent and by the Python bindings so CPU-only hosts never need
// a HIP runtime.
#pragma once

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BGC_DIAG_ABI_VERSION 11
#define BGC_DIAG_MAX_CU_KEYS 2048

typedef struct {
  uint64_t bytes;          // buffer size tested
  int iters;               // timed iterations per phase
  double write_gbps;       // pattern fill (store-only)
  double read_gbps;        // verify pass (load-only, compare in registers)
  double copy_gbps;        // device-to-device copy kernel (load+store bytes)
  uint64_t mismatches;     // words that failed the pattern check
  uint64_t first_bad_word; // index of the first failing word (UINT64_MAX if none)
  double elapsed_ms;
} bgc_hbm_result;

typedef struct {
  uint64_t tiles_checked;   // 16x16x32 bf16 MFMA tiles verified element-wise
  uint64_t mismatches;      // output elements that differed from the exact result
  int cus_seen;             // distinct (XCC, SE, SH, CU) that executed the test
  int bad_cus;              // CUs with >= 1 mismatch
  int xccs_seen;            // distinct XCC ids
  double tflops;            // dense bf16 MFMA rate of the throughput phase
  int throughput_ok;        // throughput phase accumulators matched exactly
  double elapsed_ms;
  int bad_cu_keys[64];      // first bad CU keys (xcc<<8 | se<<5 | sh<<4 | cu)
  int xcc_waves[8];         // throughput-phase waves that ran on each XCC
  double xcc_wave_us[8];    // their mean duration (constant 100 MHz clock)
  double xcc_balance;       // fastest / slowest XCC mean wave time (1.0 = balanced)
} bgc_mfma_result;

int bgc_diag_abi_version(void);
int bgc_diag_device_count(void);
// Returns 0 on success, non-zero on HIP error (message via bgc_diag_last_error()).
int bgc_diag_hbm(int device, uint64_t bytes, int iters, uint32_t seed, bgc_hbm_result* out);
int bgc_diag_mfma(int device, int waves_per_cu, int throughput_iters, uint32_t seed, bgc_mfma_result* out);
typedef struct {
  uint64_t tiles_checked;         // 16x16x128 MX tiles verified element-wise (all four variants)
  uint64_t fp8_mismatches;        // e4m3 operands, unit E8M0 scales
  uint64_t fp8_scaled_mismatches; // e4m3 operands, per-32-element-block scales in {1/2, 1, 2}
  uint64_t fp4_mismatches;        // e2m1 operands, unit scales
  uint64_t fp4_scaled_mismatches; // e2m1 operands, block scales
  int cus_seen;
  int bad_cus;                    // CUs with >= 1 mismatch in any variant
  double fp8_tflops;              // dense MX-fp8 rate (v_mfma_scale_f32_16x16x128_f8f6f4)
  double fp4_tflops;              // dense MX-fp4 rate, same instruction
  int throughput_ok;              // both rate phases' accumulators matched exactly
  double elapsed_ms;
  int bad_cu_keys[64];
} bgc_lowp_result;

// The block-scaled low-precision matrix-core path (the one fp8/fp4 inference uses), which
// the bf16 checks above never exercise: exact-integer fp8 and fp4 tiles with and without
// E8M0 block scales on every CU, then the dense fp8 and fp4 rates.
int bgc_diag_mfma_lowp(int device, int waves_per_cu, int throughput_iters, uint32_t seed, bgc_lowp_result* out);
typedef struct {
  int launches;             // throughput kernels run back to back
  double elapsed_ms;        // wall time of the burn (device events)
  double tflops_mean;       // dense bf16 MFMA rate over the whole burn
  double tflops_min;        // slowest launch
  double tflops_first;      // first launch (includes the clock ramp from idle)
  double tflops_last;       // last launch vs the best one: a drop means the GPU throttled
  double tflops_max;
  uint64_t mismatches;      // accumulator errors over all launches
} bgc_burn_result;

// Sustained MFMA load for `duration_ms` (back-to-back throughput kernels of ~10 ms each):
// the node agent samples power, clocks, temperatures and throttle residency meanwhile.
int bgc_diag_burn(int device, int duration_ms, int waves_per_cu, uint32_t seed, bgc_burn_result* out);
// The same load on another matrix-core path: BGC_BURN_FP8 / BGC_BURN_FP4 run the MX
// block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 rate kernel (rates in that dtype's FLOP/s).
#define BGC_BURN_BF16 0
#define BGC_BURN_FP8 1
#define BGC_BURN_FP4 2
int bgc_diag_burn_dtype(int device, int duration_ms, int waves_per_cu, uint32_t seed, int dtype, bgc_burn_result* out);
// C[m,n] (fp32) = A[m,k] * B[k,n], A/B bf16 bit patterns, row-major, via MFMA; the host
// compares C with its own fp32 product (m, n multiples of 16; k a multiple of 32).
int bgc_diag_gemm(int device, int m, int n, int k, const uint16_t* a_bf16, const uint16_t* b_bf16, float* c);
typedef struct {
  uint64_t bytes;           // transfer size (pinned host buffers)
  int iters;
  double h2d_gbps;          // best host -> device rate
  double d2h_gbps;          // best device -> host rate
  double bidir_gbps;        // both directions at once on two streams (sum of the two)
  uint64_t mismatches;      // 64-bit words that did not survive the H2D + D2H round trip
  double elapsed_ms;
} bgc_pcie_result;

// Host <-> device DMA over the GPU's PCIe link: a link that trained narrow or slow, or
// that replays, shows up here before a training job's data loader notices.
int bgc_diag_pcie(int device, uint64_t bytes, int iters, uint32_t seed, bgc_pcie_result* out);
typedef struct {
  int m, n, k;              // C[m,n] = A[m,k] * B[k,n], bf16 in, fp32 out
  int launches;             // back-to-back GEMMs
  double elapsed_ms;        // sum of the launches (device events)
  double tflops_mean;       // over all launches
  double tflops_best;
  uint64_t row_mismatches;  // C row sums that differ from A (B 1)  (after the first and the last launch)
  uint64_t col_mismatches;  // C column sums that differ from (1^T A) B
  int tile;                 // 256 (256x256 tile, 8 waves) or 128 (128x128, 4 waves)
  int kernel;               // 2: 8-phase ping-pong (K % 128 == 0), 1: double-buffered
} bgc_soak_result;

// GEMM soak: an LDS-tiled (global_load_lds double buffering, XOR-swizzled LDS) bf16 MFMA
// GEMM run `launches` times back to back on operands in {-1, 0, 1}, checked by exact
// row/column checksums (ABFT).  m, n multiples of 128; k a multiple of 64.
int bgc_diag_gemm_soak(int device, int m, int n, int k, int launches, uint32_t seed, bgc_soak_result* out);
// The soak's GEMM kernel on caller operands: C[m,n] (fp32) = A[m,k] * Bt[n,k]^T, A/Bt bf16
// bit patterns, row-major (so both are K-contiguous, as the kernel reads them); same shape
// rules as bgc_diag_gemm_soak.  Lets a test compare the LDS-tiled kernel on random data
// with an independent fp32 product.
int bgc_diag_gemm_tiled(int device, int m, int n, int k, const uint16_t* a_bf16, const uint16_t* bt_bf16, float* c);
// The MX block-scaled matrix-core path (v_mfma_scale_f32_16x16x128_f8f6f4) on caller
// operands: C[m,n] (fp32) = sum_k a(m,k) 2^(sa(m,k/32)-127) * bt(n,k) 2^(sb(n,k/32)-127).
// fmt 0: fp8 e4m3 (OCP), one byte per element; fmt 4: fp4 e2m1, two per byte (element 2i in
// the low nibble).  a is m x k, bt is n x k (row-major, K-contiguous), the E8M0 scales are
// m x k/32 and n x k/32 bytes.  m, n multiples of 16; k a multiple of 128.  Lets a test
// check the hardware's operand and scale layout against an independent decode.
int bgc_diag_mx_gemm(int device, int fmt, int m, int n, int k, const uint8_t* a, const uint8_t* a_scales,
                     const uint8_t* bt, const uint8_t* bt_scales, float* c);

typedef struct {
  uint64_t free_bytes;        // hipMemGetInfo before the walk
  uint64_t total_bytes;
  uint64_t target_bytes;      // fraction * free_bytes
  uint64_t bytes_covered;     // allocated and written + verified with both patterns
  int chunks;                 // device allocations the walk spans
  int passes;                 // completed passes (2 = address pattern, then its inverse)
  uint64_t mismatches;        // 64-bit words that read back wrong
  uint64_t first_bad_addr;    // device address of the lowest failing word (0 = none)
  uint64_t first_bad_xor;     // expected ^ found at that word: the flipped bits
  double write_gbps;          // fill rate over the covered bytes
  double read_gbps;           // verify rate
  double alloc_ms;            // of which: allocating the chunks
  double elapsed_ms;          // wall time of the walk (allocation included)
  int budget_hit;             // 1 when the time budget ended the walk before both passes
} bgc_hbm_walk_result;

// Pattern walk of (nearly) all free HBM: allocates `fraction` of the free VRAM in chunks of
// `chunk_bytes`, writes every 64-bit word with its own device address XOR a seed-derived
// key, verifies all of it only after every chunk was written (a write that lands on the
// wrong row or stack shows up as a wrong address elsewhere), then repeats with the inverse
// so every cell is checked holding both 0 and 1.  Stops early after `budget_ms`.
int bgc_diag_hbm_walk(int device, double fraction, uint64_t chunk_bytes, int budget_ms, uint32_t seed,
                      bgc_hbm_walk_result* out);
// PCI bus id of a HIP device ("0000:05:00.0", lower-case hex) — the key the node agent and
// the RCCL probe use to match a HIP device (renumbered inside a container) to amdsmi.
int bgc_diag_device_bdf(int device, char* buf, size_t len);
// Device name / gfx arch string, e.g. "gfx950".
int bgc_diag_device_arch(int device, char* buf, size_t len);
const char* bgc_diag_last_error(void);

#ifdef __cplusplus
}
#endif
