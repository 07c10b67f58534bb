#include <hip/hip_runtime.h>
#include <cstdint>
__global__ void add_one(float* x, int n) { int i = blockIdx.x * blockDim.x + threadIdx.x; if (i < n) x[i] += 1.0f; }
extern "C" int probe_add_one(float* x, int n, void* stream) {
  hipLaunchKernelGGL(add_one, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, n);
  return (int)hipGetLastError();
}
extern "C" int probe_runtime_version() { int v = 0; hipRuntimeGetVersion(&v); return v; }
