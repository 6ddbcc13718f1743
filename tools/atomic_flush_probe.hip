// atomic_flush_probe.hip -- cost of the end-of-kernel histogram flush: every
// workgroup of a grid adds NB counters to one u64 histogram with global
// atomics (what the round-loop kernels do once per workgroup), against the
// same adds spread over 64 copies 256 bytes apart, for several grid sizes.
// Each kernel does nothing else, so its time is the flush alone.
//   hipcc --offload-arch=gfx950 -O3 tools/atomic_flush_probe.hip -o tools/atomic_flush_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void flush_one(unsigned long long *h, int nb) {
  if (threadIdx.x < (unsigned)nb) atomicAdd(&h[threadIdx.x], 1ull);
}

__global__ void flush_spread(unsigned long long *h, int nb) {
  if (threadIdx.x < (unsigned)nb) atomicAdd(&h[(blockIdx.x & 63u) * 32u + threadIdx.x], 1ull);
}

__global__ void empty_kernel(unsigned long long *, int) {}

int main() {
  unsigned long long *h;
  hipMalloc(&h, 64 * 32 * 8);
  hipMemset(h, 0, 64 * 32 * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int grids[] = {256, 512, 1024, 2048, 4096};
  const int nbs[] = {1, 10};
  for (int warm = 0; warm < 2; ++warm)
    for (int nb : nbs)
      for (int g : grids)
        for (int k = 0; k < 3; ++k) {
          void (*fn)(unsigned long long *, int) = k == 0 ? flush_one : (k == 1 ? flush_spread : empty_kernel);
          for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(fn, dim3(g), dim3(256), 0, 0, h, nb);
          hipEventRecord(a, 0);
          for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(fn, dim3(g), dim3(256), 0, 0, h, nb);
          hipEventRecord(b, 0);
          hipEventSynchronize(b);
          float ms = 0;
          hipEventElapsedTime(&ms, a, b);
          if (warm)
            printf("{\"kernel\": \"%s\", \"grid\": %d, \"bins\": %d, \"us_per_launch\": %.3f}\n",
                   k == 0 ? "one_copy" : (k == 1 ? "64_copies" : "empty"), g, nb, ms * 1e3 / 50);
        }
  return 0;
}
