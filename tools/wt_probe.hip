// wt_probe.hip -- does a kernel's dirty L2 footprint cost its successor? (MI355X_MICROARCH "boundary":
// + B / 6 TB/s when the predecessor leaves B bytes dirty). A producer writes B bytes with plain,
// nt or sc1 (write-through) vector stores, 16 or 4 bytes per lane; a consumer reads them back (or a
// trivial kernel follows). The pair is captured 20x into a graph and replayed between two events.
//   hipcc --offload-arch=gfx950 -O3 -o tools/wt_probe tools/wt_probe.hip && tools/wt_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

enum { PLAIN = 0, NT = 1, WT = 2 };
typedef float v4f __attribute__((ext_vector_type(4)));

template <int MODE>
__device__ __forceinline__ void st16(float4* p, float4 v) {
  if constexpr (MODE == PLAIN) {
    *p = v;
  } else if constexpr (MODE == NT) {
    __builtin_nontemporal_store(v4f{v.x, v.y, v.z, v.w}, reinterpret_cast<v4f*>(p));
  } else {
    const v4f vv = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(vv) : "memory");
  }
}

template <int MODE>
__device__ __forceinline__ void st4(int* p, int v) {
  if constexpr (MODE == PLAIN) {
    *p = v;
  } else if constexpr (MODE == NT) {
    __builtin_nontemporal_store(v, p);
  } else {
    asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void writer16(float4* out, long n4, float s) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256)
    st16<MODE>(out + i, make_float4(s, s + 1.f, s + 2.f, (float)i));
}

template <int MODE>
__global__ __launch_bounds__(256) void writer4(int* out, long n, int s) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) st4<MODE>(out + i, s + (int)i);
}

__global__ __launch_bounds__(256) void reader16(const float4* in, long n4, float* sink) {
  float acc = 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const float4 v = in[i];
    acc += v.x + v.w;
  }
  if (acc == 1234.5f) sink[0] = acc;
}

__global__ void trivial(float* sink) {
  if (threadIdx.x == 1000) sink[0] = 1.f;
}

template <typename F>
float time_graph(F body, hipStream_t st, int reps = 20, int replays = 10) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int i = 0; i < reps; ++i) body();
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, st));
  CK(hipStreamSynchronize(st));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, st));
  for (int i = 0; i < replays; ++i) CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return 1000.f * ms / (reps * replays);
}

int main() {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const long maxb = 64l << 20;
  float4* buf;
  float* sink;
  CK(hipMalloc(&buf, maxb));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(buf, 0, maxb));
  const long sizes[] = {1l << 20, 4l << 20, 12l << 20, 32l << 20};
  const char* mn[] = {"plain", "nt", "sc1"};
  printf("bytes_MB mode  w16  w16+triv  w16+read  w4  w4+triv  w4+read  (us per pair, graph of 20)\n");
  for (long B : sizes) {
    const long n4 = B / 16, n = B / 4;
    const int grid = 2048;
    for (int m = 0; m < 3; ++m) {
      auto w16 = [&] {
        if (m == 0) hipLaunchKernelGGL(writer16<PLAIN>, dim3(grid), dim3(256), 0, st, buf, n4, 1.f);
        else if (m == 1) hipLaunchKernelGGL(writer16<NT>, dim3(grid), dim3(256), 0, st, buf, n4, 1.f);
        else hipLaunchKernelGGL(writer16<WT>, dim3(grid), dim3(256), 0, st, buf, n4, 1.f);
      };
      auto w4 = [&] {
        int* ib = reinterpret_cast<int*>(buf);
        if (m == 0) hipLaunchKernelGGL(writer4<PLAIN>, dim3(grid), dim3(256), 0, st, ib, n, 1);
        else if (m == 1) hipLaunchKernelGGL(writer4<NT>, dim3(grid), dim3(256), 0, st, ib, n, 1);
        else hipLaunchKernelGGL(writer4<WT>, dim3(grid), dim3(256), 0, st, ib, n, 1);
      };
      auto tr = [&] { hipLaunchKernelGGL(trivial, dim3(256), dim3(256), 0, st, sink); };
      auto rd = [&] { hipLaunchKernelGGL(reader16, dim3(grid), dim3(256), 0, st, buf, n4, sink); };
      const float a = time_graph([&] { w16(); }, st);
      const float b = time_graph([&] { w16(); tr(); }, st);
      const float c = time_graph([&] { w16(); rd(); }, st);
      const float d = time_graph([&] { w4(); }, st);
      const float e = time_graph([&] { w4(); tr(); }, st);
      const float f = time_graph([&] { w4(); rd(); }, st);
      printf("%6.0f %-5s %7.2f %7.2f %7.2f %7.2f %7.2f %7.2f\n", B / 1048576.0, mn[m], a, b, c, d, e, f);
      fflush(stdout);
    }
  }
  const float t = time_graph([&] { hipLaunchKernelGGL(trivial, dim3(256), dim3(256), 0, st, sink); }, st);
  printf("trivial alone %.2f us\n", t);
  return 0;
}
