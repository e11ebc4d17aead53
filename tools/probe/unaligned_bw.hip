// Probe: bandwidth of a coalesced 16-byte copy (consecutive lanes,
// consecutive chunks -- the shape of the var encode's payload chunk map)
// when the source is byte/word misaligned, vs aligned loads + a funnel
// shift with the neighbouring lane's chunk.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_copy16(const uint8_t *in, uint8_t *out, long n, int sh_in) {
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i < n) {
    u32x4 v = *reinterpret_cast<const u32x4 *>(in + sh_in + 16 * i);
    *reinterpret_cast<u32x4 *>(out + 16 * i) = v;
  }
}
// aligned loads; bytes [16i+sh, 16i+sh+16) from this lane's chunk and the next lane's
__global__ void k_copy16_shfl(const uint8_t *in, uint8_t *out, long n, int sh_in) {
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i < n) {
    const int sb = sh_in & 15;
    const uint8_t *base = in + (sh_in & ~15);
    u32x4 a = *reinterpret_cast<const u32x4 *>(base + 16 * i);
    u32x4 b;
    b.x = __shfl_down(a.x, 1, 64);
    b.y = __shfl_down(a.y, 1, 64);
    b.z = __shfl_down(a.z, 1, 64);
    b.w = __shfl_down(a.w, 1, 64);
    if ((threadIdx.x & 63) == 63) b = *reinterpret_cast<const u32x4 *>(base + 16 * i + 16);
    uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const int q = sb >> 2, s8 = (sb & 3) * 8;
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (j == q) { lo = w[k + j]; hi = w[k + j + 1]; }
      o[k] = s8 ? __builtin_amdgcn_alignbyte(hi, lo, sb & 3) : lo;
    }
    *reinterpret_cast<u32x4 *>(out + 16 * i) = u32x4{o[0], o[1], o[2], o[3]};
  }
}

int main() {
  const long n = 1l << 24;  // 256 MiB
  uint8_t *a, *b;
  hipMalloc(&a, 16 * n + 64);
  hipMalloc(&b, 16 * n + 64);
  hipMemset(a, 1, 16 * n + 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int variant = 0; variant < 2; ++variant)
    for (int sh : {0, 1, 2, 4, 8}) {
      auto go = [&] {
        if (variant == 0) k_copy16<<<n / 256, 256>>>(a, b, n, sh);
        else k_copy16_shfl<<<n / 256, 256>>>(a, b, n, sh);
      };
      for (int w = 0; w < 3; ++w) go();
      hipEventRecord(e0);
      for (int w = 0; w < 20; ++w) go();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      ms /= 20;
      printf("%s sh=%d: %.3f ms  %.0f GB/s\n", variant ? "shfl  " : "copy16", sh, ms, 2.0 * 16 * n / ms / 1e6);
    }
  return 0;
}
