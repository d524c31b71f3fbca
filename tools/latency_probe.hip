// Dependent-access latencies at the start of a kernel on MI355X (kernel studies, not product code):
// what a fused conv kernel's prologue chain is made of. Each launch is captured in a HIP graph after a
// 512 MB write (so the kernel arguments and the data miss L2 and the 256 MB last-level cache, as in a
// training step whose previous launches streamed other tensors), or without it (warm).
//   hipcc --offload-arch=gfx950 -O3 -o tools/latency_probe tools/latency_probe.hip && tools/latency_probe
// Per workgroup, thread 0 stamps s_memrealtime (100 MHz):
//   t0 kernel entry, t1 a kernel argument in an SGPR (scalar load from the kernarg segment),
//   t2 a scalar load through that pointer, t3 a vector load through it, t4 a second kernarg line,
//   t5 a scalar load that depends on t2's value, t6 a vector load issued at entry from the kernarg
//   segment pointer itself (no scalar wait first)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

struct Args {
  const int* p0;        // kernarg line 0
  char pad[120];
  const int* p1;        // kernarg line 2 (offset 128)
  unsigned long long* out;
};

__global__ void probe(Args a) {
  unsigned long long t[8];
  t[0] = __builtin_amdgcn_s_memrealtime();
  const int* p = a.p0;
  asm volatile("" : "+s"(p));
  t[1] = __builtin_amdgcn_s_memrealtime();
  typedef __attribute__((address_space(4))) const int cint;
  int v = *(cint*)p;  // scalar load (constant address space, uniform address)
  asm volatile("" : "+s"(v));
  t[2] = __builtin_amdgcn_s_memrealtime();
  int w = __builtin_nontemporal_load(p + 64 + (int)threadIdx.x);  // vector load
  asm volatile("" : "+v"(w));
  t[3] = __builtin_amdgcn_s_memrealtime();
  const int* q = a.p1;
  asm volatile("" : "+s"(q));
  t[4] = __builtin_amdgcn_s_memrealtime();
  int u = ((cint*)q)[v & 1023];  // scalar load depending on the previous value
  asm volatile("" : "+s"(u));
  t[5] = __builtin_amdgcn_s_memrealtime();
  t[6] = (unsigned long long)(v + w + u);
  if (threadIdx.x == 0) {
    unsigned long long* o = a.out + (size_t)blockIdx.x * 8;
    for (int i = 0; i < 7; ++i) o[i] = t[i];
  }
}

__global__ void flush(float* b, size_t n, float v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = v;
}

int main() {
  const int nwg = 256;
  int *d0, *d1;
  unsigned long long* out;
  float* fb;
  const size_t nf = (size_t)1 << 27;
  hipMalloc(&d0, 1 << 20);
  hipMalloc(&d1, 1 << 20);
  hipMemset(d0, 0, 1 << 20);
  hipMemset(d1, 0, 1 << 20);
  hipMalloc(&out, nwg * 8 * sizeof(unsigned long long));
  hipMalloc(&fb, nf * sizeof(float));
  hipStream_t s;
  hipStreamCreate(&s);
  Args a{};
  a.p0 = d0;
  a.p1 = d1;
  a.out = out;
  for (int cold = 0; cold < 2; ++cold) {
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    if (cold) hipLaunchKernelGGL(flush, dim3(4096), dim3(256), 0, s, fb, nf, 1.0f);
    hipLaunchKernelGGL(probe, dim3(nwg), dim3(256), 0, s, a);
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    std::vector<std::vector<double>> d(6);
    for (int rep = 0; rep < 20; ++rep) {
      hipGraphLaunch(ge, s);
      hipStreamSynchronize(s);
      std::vector<unsigned long long> h(nwg * 8);
      hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost);
      if (rep < 2) continue;
      for (int w = 0; w < nwg; ++w)
        for (int i = 1; i < 6; ++i) d[i].push_back((h[w * 8 + i] - h[w * 8 + i - 1]) * 0.01);
    }
    const char* nm[6] = {"", "kernarg line 0 (scalar)", "scalar load via it", "vector load via it",
                         "kernarg line 2 (scalar)", "dependent scalar load"};
    printf("%s\n", cold ? "cold (512 MB written first, in the same graph)" : "warm (graph replayed alone)");
    for (int i = 1; i < 6; ++i) {
      std::sort(d[i].begin(), d[i].end());
      printf("  %-26s med %5.2f us  p90 %5.2f us\n", nm[i], d[i][d[i].size() / 2], d[i][d[i].size() * 9 / 10]);
    }
  }
  return 0;
}
