// Exhaustive device check of the fast correctly rounded reciprocal (include/hrt/hd_math.h rcp_rn): for every f32 bit
// pattern, v_rcp_f32 followed by one fma Newton correction against IEEE 1.0f / x, on the MI355X itself.
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -Iinclude tests/native/rcp_check.hip -o rcp_check
// Prints the mismatch count per biased exponent of x (255 classes); rcp_rn's fast domain must show none.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

__global__ void check(unsigned long long* bad, unsigned int* first) {
  const unsigned long long n = 1ull << 32;
  for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
       i += (unsigned long long)gridDim.x * blockDim.x) {
    const unsigned int u = (unsigned int)i;
    const float x = __uint_as_float(u);
    const unsigned int e = (u >> 23) & 255u;
    if (e == 255u) continue; /* inf / NaN */
    const float y = __builtin_amdgcn_rcpf(x);
    const float r = __builtin_fmaf(-x, y, 1.0f);
    const float q = __builtin_fmaf(r, y, y);
    const float ieee = 1.0f / x;
    if (__float_as_uint(q) != __float_as_uint(ieee)) {
      atomicAdd(&bad[e], 1ull);
      atomicCAS(&first[e], 0xFFFFFFFFu, u);
    }
  }
}

int main() {
  unsigned long long* bad;
  unsigned int* first;
  hipMalloc(&bad, 256 * sizeof(unsigned long long));
  hipMalloc(&first, 256 * sizeof(unsigned int));
  hipMemset(bad, 0, 256 * sizeof(unsigned long long));
  hipMemset(first, 0xFF, 256 * sizeof(unsigned int));
  hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, 0, bad, first);
  hipError_t err = hipDeviceSynchronize();
  if (err != hipSuccess) {
    printf("hip error %s\n", hipGetErrorString(err));
    return 2;
  }
  unsigned long long h[256];
  unsigned int fu[256];
  hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost);
  hipMemcpy(fu, first, sizeof(fu), hipMemcpyDeviceToHost);
  unsigned long long total = 0;
  int lo = -1, hi = -1;
  for (int e = 0; e < 255; e++) {
    total += h[e];
    if (h[e] == 0 && lo < 0 && e > 0) lo = e;
    if (h[e]) {
      float x;
      memcpy(&x, &fu[e], 4);
      printf("biased exponent %3d: %llu mismatches (first x = %a)\n", e, h[e], x);
    }
  }
  for (int e = 1; e < 255; e++) if (h[e] == 0) hi = e;
  printf("total mismatches %llu over 2^32 - 2^24 finite inputs\n", total);
  return 0;
}
