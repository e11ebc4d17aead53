// Probe: s_memtime rate (vs s_memrealtime, 100 MHz) and the latency of a
// dependent global load (L2 hit / HBM miss) and of an LDS round trip, in
// s_memtime ticks -- the unit of tools/tune/enc_stamps.py.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

__global__ void k_clock(unsigned long long *out, const uint32_t *chain, uint32_t steps, uint32_t hot) {
  __shared__ uint32_t lds[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = (i * 37 + 1) & 1023;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  float x = threadIdx.x;
  for (int i = 0; i < 200000; ++i) x = x * 0.999f + 1.0f;
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  // dependent global loads
  uint32_t p = 0;
  for (uint32_t i = 0; i < hot; ++i) p = chain[p];  // warm
  unsigned long long t2 = __builtin_amdgcn_s_memtime();
  for (uint32_t i = 0; i < steps; ++i) p = chain[p];
  unsigned long long t3 = __builtin_amdgcn_s_memtime();
  // dependent LDS loads
  uint32_t q = threadIdx.x;
  for (int i = 0; i < 1000; ++i) q = lds[q];
  unsigned long long t4 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[0] = t1 - t0;
    out[1] = r1 - r0;
    out[2] = t3 - t2;
    out[3] = t4 - t3;
    out[4] = static_cast<unsigned long long>(x) + p + q;
  }
}

int main() {
  // a random cycle over 256 MiB (HBM misses) and one over 64 KiB (cache hits)
  for (size_t words : {size_t(64) << 20, size_t(16) << 10}) {
    std::vector<uint32_t> h(words);
    std::vector<uint32_t> perm(words);
    for (size_t i = 0; i < words; ++i) perm[i] = uint32_t(i);
    uint64_t s = 88172645463325252ull;
    for (size_t i = words - 1; i > 0; --i) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      std::swap(perm[i], perm[s % (i + 1)]);
    }
    for (size_t i = 0; i < words; ++i) h[perm[i]] = perm[(i + 1) % words];
    uint32_t *d;
    unsigned long long *o;
    hipMalloc(&d, words * 4);
    hipMalloc(&o, 64);
    hipMemcpy(d, h.data(), words * 4, hipMemcpyHostToDevice);
    const uint32_t steps = 2000;
    k_clock<<<1, 64>>>(o, d, steps, words < 100000 ? 20000 : 0);
    unsigned long long r[5];
    hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
    printf("chain %zu KiB: s_memtime/s_memrealtime = %.2f (=> s_memtime %.0f MHz); dependent load %.0f ticks; LDS RT %.0f ticks\n",
           words * 4 / 1024, double(r[0]) / r[1], 100.0 * r[0] / r[1], double(r[2]) / steps, double(r[3]) / 1000);
    hipFree(d);
    hipFree(o);
  }
  return 0;
}
