// Which lane's E8M0 scale byte v_mfma_scale_f32_16x16x128_f8f6f4 applies to each of a
// lane group's 32 operand elements, for fp8 (fmt 0) and fp4 (fmt 4).  One wave per
// element position p = 32 g + j: only A row 0's element j of lane group g is 1.0, B is all
// ones with unit scales, and lane group g' supplies scale 2^(g' + 1).  C[0][0] is then the
// scale that hit that element; log2 - 1 names the lane group it came from.
//   hipcc --offload-arch=gfx950 -O2 tools/probes/mx_scale_layout.hip -o tools/probes/mx_scale_layout
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int kFmt>
__global__ __launch_bounds__(64) void probe(float* out) {
  const int lane = threadIdx.x, p = blockIdx.x, g0 = p / 32, j0 = p % 32;
  const unsigned one = kFmt == 0 ? 0x38u : 0x2u;
  i32x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, b = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = 0; j < 32; ++j) {
    const int sh = kFmt == 0 ? 8 * (j & 3) : 4 * (j & 7);
    const int w = kFmt == 0 ? j >> 2 : j >> 3;
    b[w] |= static_cast<int>(one << sh);
    if ((lane & 15) == 0 && (lane >> 4) == g0 && j == j0) a[w] |= static_cast<int>(one << sh);
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, kFmt, kFmt, 0, 128 + (lane >> 4), 0, 127);
  out[p * 64 + lane] = acc[0];  // every lane stores: a lane-0-only store lets the compiler sink the MFMA under that branch
}

int main() {
  float* d = nullptr;
  static float h[128 * 64];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
  for (int fmt = 0; fmt < 2; ++fmt) {
    if (fmt == 0) {
      hipLaunchKernelGGL(probe<0>, dim3(128), dim3(64), 0, nullptr, d);
    } else {
      hipLaunchKernelGGL(probe<4>, dim3(128), dim3(64), 0, nullptr, d);
    }
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    std::printf("{\"fmt\": \"%s\", \"scale_group\": [", fmt == 0 ? "fp8" : "fp4");
    for (int p = 0; p < 128; ++p) {
      const float v = h[p * 64];  // lane 0: C[0][0]
      const int grp = v > 0 ? static_cast<int>(std::lround(std::log2(v))) - 1 : -9;
      std::printf("%s%d", p ? ", " : "", grp);
    }
    std::printf("]}\n");
  }
  (void)hipFree(d);
  return 0;
}
