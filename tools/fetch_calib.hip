// Profiling-only: calibrate rocprofv3 FETCH_SIZE against a known byte count for the read
// patterns of the step kernel (MI355X_MICROARCH.md §HBM: the 1/2 factor is established for
// 16-B-per-lane streaming reads only).  Each kernel reads `bytes` once from a 1 GiB buffer
// (past the 256 MiB Infinity Cache) and writes one float per wave.
//   dword32: 32 active lanes x 4 B per wave-instruction (the step kernel's SoA channel loads)
//   dword64: 64 lanes x 4 B
//   qword32: 32 lanes x 8 B (progress / reset int64)
//   f4_64:   64 lanes x 16 B (actions, obs-sized streams)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <typename T, int LANES>
__global__ __launch_bounds__(64) void rd(const T* __restrict__ src, int64_t n_per_wave, float* out) {
  const int lane = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * n_per_wave;
  float acc = 0.0f;
  if (lane < LANES)
    for (int64_t i = lane; i < n_per_wave; i += LANES) {
      T v = src[base + i];
      acc += *reinterpret_cast<const float*>(&v);
    }
  if (lane == 0) out[blockIdx.x] = acc;
}

int main() {
  const size_t bytes = size_t(1) << 30;
  char* buf;
  float* out;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
  if (hipMemset(buf, 0, bytes) != hipSuccess) return 1;
  const int waves = 8192;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL((rd<float, 32>), dim3(waves), dim3(64), 0, 0, (const float*)buf, (int64_t)(bytes / 4 / waves), out);
    hipLaunchKernelGGL((rd<float, 64>), dim3(waves), dim3(64), 0, 0, (const float*)buf, (int64_t)(bytes / 4 / waves), out);
    hipLaunchKernelGGL((rd<double, 32>), dim3(waves), dim3(64), 0, 0, (const double*)buf, (int64_t)(bytes / 8 / waves), out);
    hipLaunchKernelGGL((rd<float4, 64>), dim3(waves), dim3(64), 0, 0, (const float4*)buf, (int64_t)(bytes / 16 / waves), out);
  }
  hipDeviceSynchronize();
  printf("read %zu bytes per dispatch\n", bytes);
  return 0;
}
