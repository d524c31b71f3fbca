// icache_probe.hip -- cost of long straight-line kernels (kernel studies; not product code)
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int N, int LOOP>
__global__ __launch_bounds__(256) void k(float* out, float s) {
  float a = threadIdx.x * s, b = a + 1.f, c = a + 2.f, d = a + 3.f;
  for (int l = 0; l < LOOP; ++l) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      a = a * 1.0001f + (float)(i + 1);
      b = b * 0.9999f + (float)(i + 3);
      c = c * 1.0002f + (float)(i + 5);
      d = d * 0.9998f + (float)(i + 7);
    }
  }
  if (a + b + c + d == 1234.5f) out[threadIdx.x] = a;
}
template <int N, int LOOP>
void run(float* o, int blocks, hipStream_t st) {
  hipGraph_t g; hipGraphExec_t ge;
  hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
  for (int r = 0; r < 20; ++r) hipLaunchKernelGGL((k<N, LOOP>), dim3(blocks), dim3(256), 0, st, o, 1.0f);
  hipStreamEndCapture(st, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, st);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, st);
  for (int i = 0; i < 10; ++i) hipGraphLaunch(ge, st);
  hipEventRecord(e1, st); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("unrolled %5d x loop %3d (VALU/wave %6d)  blocks %4d: %7.2f us\n", N * 8, LOOP, N * 8 * LOOP, blocks, 1000.f * ms / 200);
}
int main() {
  float* o; hipMalloc(&o, 4096); hipStream_t st; hipStreamCreate(&st);
  for (int b : {256, 1024}) {
    run<16, 1>(o, b, st);
    run<16, 16>(o, b, st);
    run<256, 1>(o, b, st);
    run<16, 64>(o, b, st);
    run<1024, 1>(o, b, st);
  }
}
