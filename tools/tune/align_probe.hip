// Read rate of 16-byte global loads by source alignment: every lane reads
// consecutive 16-byte pieces starting at byte `off` of a 1 GiB buffer and
// writes one word per lane (so the loads are not dropped).  Modes:
//   0 one dwordx4 load at base+off            (off 0: aligned; 4: dword; 1: byte)
//   1 dword-aligned dwordx4 + one dword, alignbyte  (the one-pass encode's form)
//   2 two aligned dwordx4 and a byte funnel
//   hipcc --offload-arch=gfx950 -O3 -o tools/tune/_align_probe tools/tune/align_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void rd(const uint8_t *__restrict__ p, uint64_t n16, uint32_t off, uint32_t *out) {
  uint32_t acc = 0;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256u;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += stride) {
    const uint64_t a = i * 16u + off;
    if constexpr (MODE == 0) {
      const u4 t = *reinterpret_cast<const u4 *>(p + a);
      acc += t.x ^ t.y ^ t.z ^ t.w;
    } else if constexpr (MODE == 1) {
      const uint64_t a4 = a & ~3ull;
      const uint32_t sb = a & 3u;
      const u4 t = *reinterpret_cast<const u4 *>(p + a4);
      const uint32_t t4 = sb ? *reinterpret_cast<const uint32_t *>(p + a4 + 16) : 0u;
      acc += __builtin_amdgcn_alignbyte(t.y, t.x, sb) ^ __builtin_amdgcn_alignbyte(t.z, t.y, sb) ^
             __builtin_amdgcn_alignbyte(t.w, t.z, sb) ^ __builtin_amdgcn_alignbyte(t4, t.w, sb);
    } else {
      const uint64_t a16 = a & ~15ull;
      const uint32_t sh = a & 15u;
      const u4 t = *reinterpret_cast<const u4 *>(p + a16);
      const u4 v = *reinterpret_cast<const u4 *>(p + a16 + 16);
      const uint32_t w[8] = {t.x, t.y, t.z, t.w, v.x, v.y, v.z, v.w};
      const uint32_t q = sh >> 2, sb = sh & 3u;
      uint32_t r = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        uint32_t lo = w[k], hi = w[k + 1];
#pragma unroll
        for (int j = 1; j < 4; ++j) {
          lo = q == static_cast<uint32_t>(j) ? w[k + j] : lo;
          hi = q == static_cast<uint32_t>(j) ? w[k + j + 1] : hi;
        }
        r ^= __builtin_amdgcn_alignbyte(hi, lo, sb);
      }
      acc += r;
    }
  }
  out[blockIdx.x * 256u + threadIdx.x] = acc;
}

int main() {
  const uint64_t bytes = 1ull << 30;
  uint8_t *p;
  uint32_t *o;
  hipMalloc(&p, bytes + 64);
  hipMemset(p, 1, bytes + 64);
  const int grid = 256 * 16;
  hipMalloc(&o, grid * 256 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const uint64_t n16 = bytes / 16;
  for (int mode = 0; mode < 3; ++mode)
    for (uint32_t off : {0u, 4u, 1u, 7u}) {
      float best = 1e9f;
      for (int rep = 0; rep < 6; ++rep) {
        hipEventRecord(e0);
        if (mode == 0) rd<0><<<grid, 256>>>(p, n16, off, o);
        else if (mode == 1) rd<1><<<grid, 256>>>(p, n16, off, o);
        else rd<2><<<grid, 256>>>(p, n16, off, o);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep && ms < best) best = ms;
      }
      printf("mode %d off %u: %.3f ms  %.2f TB/s\n", mode, off, best, bytes / (best * 1e-3) / 1e12);
    }
  return hipDeviceSynchronize() != hipSuccess;
}
