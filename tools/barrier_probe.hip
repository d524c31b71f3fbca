// barrier_probe.hip -- cost of an in-launch barrier across P workgroups ("a barrier
// across <= 32 workgroups on one XCD against the 1.45 us kernel boundary").
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/barrier_probe tools/barrier_probe.hip && tools/barrier_probe
//
// Grid: 256 workgroups of 256 threads, one per CU (all resident). Participants:
//   xcd0_32 : the 32 workgroups of XCD 0 (blockIdx % 8 == 0 -- round-robin dispatch over the 8 XCDs)
//   spread_32: blockIdx < 32 (4 per XCD)
//   all_256 : every workgroup
// The rest exit at once. Barrier: one monotonic device-scope counter per variant; lane 0 arrives with a
// release fetch_add and polls relaxed (s_sleep between polls), then an acquire fence and the workgroup
// barrier. R rounds; each participant stamps s_memrealtime (100 MHz) before the first and after the last
// round, so the per-barrier cost = (t1 - t0) / R, max over participants. Every poll loop is bounded (an
// error flag instead of a hang).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ __launch_bounds__(256) void barrier_kernel(unsigned* cnt, int mode, int rounds, unsigned long long* t,
                                                      int* err) {
  const int b = blockIdx.x;
  const bool part = mode == 0 ? (b % 8 == 0) : mode == 1 ? (b < 32) : true;
  if (!part) return;
  const unsigned P = mode == 2 ? 256u : 32u;
  const int slot = mode == 0 ? b / 8 : b;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int r = 0; r < rounds; ++r) {
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = P * (unsigned)(r + 1);
      int polls = 0;
      while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++polls > 2000000) {
          atomicAdd(err, 1);
          break;
        }
      }
      __atomic_thread_fence(__ATOMIC_ACQUIRE);
    }
    __syncthreads();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    t[2 * slot] = t0;
    t[2 * slot + 1] = t1;
  }
}

__global__ void empty_kernel(int* p) {
  if (threadIdx.x == 0 && p[0] == 12345) p[1] = 1;
}

int main() {
  const int rounds = 2000;
  unsigned* cnt;
  unsigned long long* t;
  int* err;
  (void)hipMalloc(&cnt, 4);
  (void)hipMalloc(&t, 2 * 256 * 8);
  (void)hipMalloc(&err, 8);
  const char* names[3] = {"xcd0_32", "spread_32", "all_256"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipMemset(cnt, 0, 4);
      (void)hipMemset(t, 0, 2 * 256 * 8);
      (void)hipMemset(err, 0, 8);
      hipLaunchKernelGGL(barrier_kernel, dim3(256), dim3(256), 0, 0, cnt, mode, rounds, t, err);
      (void)hipDeviceSynchronize();
      std::vector<unsigned long long> h(512);
      int e = 0;
      (void)hipMemcpy(h.data(), t, 512 * 8, hipMemcpyDeviceToHost);
      (void)hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
      const int np = mode == 2 ? 256 : 32;
      unsigned long long lo = ~0ull, hi = 0;
      for (int i = 0; i < np; ++i) {
        if (h[2 * i] < lo) lo = h[2 * i];
        if (h[2 * i + 1] > hi) hi = h[2 * i + 1];
      }
      printf("%-10s rep %d: %.3f us per barrier (%d rounds, %d participants, errors %d)\n", names[mode], rep,
             (double)(hi - lo) * 0.01 / rounds, rounds, np, e);
    }
  }
  // kernel boundary: K dependent empty launches in a captured graph, replayed
  int* p;
  (void)hipMalloc(&p, 8);
  (void)hipMemset(p, 0, 8);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  for (int grid : {32, 256}) {
    const int K = 200;
    hipGraph_t g;
    hipGraphExec_t ge;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int k = 0; k < K; ++k) hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(256), 0, s, p);
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    (void)hipGraphLaunch(ge, s);
    (void)hipStreamSynchronize(s);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, s);
    for (int it = 0; it < 10; ++it) (void)hipGraphLaunch(ge, s);
    (void)hipEventRecord(e1, s);
    (void)hipStreamSynchronize(s);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("boundary   grid %3d: %.3f us per empty launch in a replayed graph (%d launches x 10)\n", grid,
           ms * 1000.0 / (10 * K), K);
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
  }
  return 0;
}
