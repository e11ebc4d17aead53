// Kernels with private (scratch) memory for tools/gpu/graph_node_probe.py:
// does a captured kernel that uses scratch replay correctly, alone and when
// an uncaptured launch between replays makes the runtime grow its scratch?
// Built by the probe itself (hipcc --genco, gfx950); not part of the product.
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int N>
__device__ __forceinline__ void scratch_body(uint32_t *out, uint32_t n, uint32_t k) {
  uint32_t a[N];  // dynamically indexed: lives in private memory
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  for (uint32_t i = 0; i < N; ++i) a[(i * k + t) & (N - 1)] = i ^ t;
  uint32_t s = 0;
  for (uint32_t i = 0; i < N; ++i) s += a[(i * 7u + t) & (N - 1)] * (i + 1);
  if (t < n) out[t] = s;
}

extern "C" __global__ void __launch_bounds__(256) scratch_small(uint32_t *out, uint32_t n, uint32_t k) {
  scratch_body<64>(out, n, k);
}

extern "C" __global__ void __launch_bounds__(256) scratch_big(uint32_t *out, uint32_t n, uint32_t k) {
  scratch_body<2048>(out, n, k);
}
