// Minimal repro for rocprofv3's exit-time SIGSEGV after a cooperative launch (docs/PERF.md):
// one trivial kernel launched with hipLaunchCooperativeKernel, nothing else.  Run plain and
// under `rocprofv3 --kernel-trace --stats -- ./coop_repro [coop=1|0]`.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void touch(int* p) {
  if (threadIdx.x == 0) p[blockIdx.x] = blockIdx.x;
}

int main(int argc, char** argv) {
  const bool coop = argc < 2 || std::atoi(argv[1]) != 0;
  int* d = nullptr;
  if (hipMalloc(&d, 256 * sizeof(int)) != hipSuccess) return 2;
  void* args[] = {&d};
  hipError_t e = coop ? hipLaunchCooperativeKernel((const void*)touch, dim3(256), dim3(512), args, 0, nullptr)
                      : hipLaunchKernel((const void*)touch, dim3(256), dim3(512), args, 0, nullptr);
  if (e != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    std::printf("launch failed: %s\n", hipGetErrorString(e));
    return 3;
  }
  int h[256];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 4;
  int bad = 0;
  for (int i = 0; i < 256; ++i) bad += h[i] != i;
  (void)hipFree(d);
  std::printf("coop=%d bad=%d\n", coop ? 1 : 0, bad);
  return bad ? 1 : 0;
}
