// Profiling-only: calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE against known byte counts for the
// access patterns of the step kernel (MI355X_MICROARCH.md §HBM: FETCH_SIZE's 1/2 factor and
// WRITE_SIZE's exactness are established for 16-B-per-lane streams only).  Each `rd` kernel reads
// `bytes` once from a 1 GiB buffer (past the 256 MiB Infinity Cache) and writes one float per wave;
// each `wr` kernel writes `bytes` once.
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

template <typename T, int LANES>
__global__ __launch_bounds__(64) void wr(T* __restrict__ dst, int64_t n_per_wave) {
  const int lane = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * n_per_wave;
  if (lane < LANES)
    for (int64_t i = lane; i < n_per_wave; i += LANES) dst[base + i] = T{};
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
    //   writes: dword32 (SoA state), byte64 (time_outs), qword32 (int64 bookkeeping), f4_64 (obs)
    hipLaunchKernelGGL((wr<float, 32>), dim3(waves), dim3(64), 0, 0, (float*)buf, (int64_t)(bytes / 4 / waves));
    hipLaunchKernelGGL((wr<unsigned char, 64>), dim3(waves), dim3(64), 0, 0, (unsigned char*)buf, (int64_t)(bytes / waves));
    hipLaunchKernelGGL((wr<double, 32>), dim3(waves), dim3(64), 0, 0, (double*)buf, (int64_t)(bytes / 8 / waves));
    hipLaunchKernelGGL((wr<float4, 64>), dim3(waves), dim3(64), 0, 0, (float4*)buf, (int64_t)(bytes / 16 / waves));
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("read or wrote %zu bytes per dispatch\n", bytes);
  return 0;
}
