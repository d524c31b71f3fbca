// fetch_cal.hip -- calibrate rocprofv3's FETCH_SIZE on gfx950 for the load widths this path uses
// (MI355X_MICROARCH "HBM": FETCH_SIZE is 1/2 of a 16-B-per-lane streaming read; other widths
// uncalibrated). Each kernel streams 64 MiB once with 16-, 8-, 4- or 1-byte loads per lane (a wave
// covers contiguous bytes) and writes one value per workgroup; run it under
//   rocprofv3 --pmc FETCH_SIZE -- tools/fetch_cal
// and divide each kernel's FETCH_SIZE (KB) by 65536 KB.
//   hipcc --offload-arch=gfx950 -O3 -o tools/fetch_cal tools/fetch_cal.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

template <typename T>
__global__ __launch_bounds__(256) void read_kernel(const T* __restrict__ in, long n, float* sink) {
  float acc = 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const T v = in[i];
    acc += (float)(reinterpret_cast<const unsigned char*>(&v)[0]);
  }
  if (acc == -1.f) sink[blockIdx.x] = acc;
}

int main() {
  const long bytes = 64l << 20;
  void* buf;
  float* sink;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 1 << 20) != hipSuccess) return 1;
  (void)hipMemset(buf, 1, bytes);
  const dim3 g(4096), b(256);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(read_kernel<int4>, g, b, 0, 0, (const int4*)buf, bytes / 16, sink);
    hipLaunchKernelGGL(read_kernel<int2>, g, b, 0, 0, (const int2*)buf, bytes / 8, sink);
    hipLaunchKernelGGL(read_kernel<int>, g, b, 0, 0, (const int*)buf, bytes / 4, sink);
    hipLaunchKernelGGL(read_kernel<char>, g, b, 0, 0, (const char*)buf, bytes, sink);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("streamed %ld bytes per kernel (int4, int2, int, char), twice\n", bytes);
  return 0;
}
