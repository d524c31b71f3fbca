#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v2i __attribute__((ext_vector_type(2)));
// LDS bytes: lds[i] = i (16-bit ids split in two passes). Lane l reads with address off(l).
__global__ void probe(int* out, int mode, int hi) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[8192];
  for (int i = threadIdx.x; i < 8192; i += 64) lds[i] = hi ? (unsigned char)(i >> 8) : (unsigned char)i;
  __syncthreads();
  const int l = threadIdx.x;
  int off;
  if (mode == 0) off = l * 8;                 // each lane: its own 8-byte chunk, contiguous
  else if (mode == 1) off = l * 16;           // 16-byte stride
  else off = (l & 15) * 64 + (l >> 4) * 8;    // rows of 64 B
  v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(lds + off));
  out[l * 2] = v.x;
  out[l * 2 + 1] = v.y;
}
int main() {
  int* d;
  hipMalloc(&d, 128 * 4);
  int h[128], hh[128];
  for (int mode = 0; mode < 3; ++mode) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, mode, 0);
    hipMemcpy(h, d, 128 * 4, hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, mode, 1);
    hipMemcpy(hh, d, 128 * 4, hipMemcpyDeviceToHost);
    printf("mode %d\n", mode);
    for (int l = 0; l < 64; ++l) {
      printf("lane %2d:", l);
      for (int j = 0; j < 8; ++j) {
        const int w = j / 4, b = j % 4;
        const int lo = (h[l * 2 + w] >> (8 * b)) & 0xff, hi = (hh[l * 2 + w] >> (8 * b)) & 0xff;
        printf(" %4d", hi * 256 + lo);
      }
      printf("\n");
    }
  }
  return 0;
}
