// Tuning harness (not part of the product): sweeps the template and launch
// parameters of k_fixed_reg against a plain 16-byte copy with the same
// access pattern, all in one process so variants are compared interleaved.
#include "../../xdrpp_amd/csrc/kernels.h"

using namespace xdrg;
using namespace xdrg::dev;

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy(const u32x4 *__restrict__ in, u32x4 *__restrict__ out,
                                              uint64_t n) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t c = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; c < n; c += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (c + u * stride < n) v[u] = NT ? __builtin_nontemporal_load(in + c + u * stride) : in[c + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (c + u * stride < n) {
        if (NT) __builtin_nontemporal_store(v[u], out + c + u * stride); else out[c + u * stride] = v[u];
      }
  }
}

#define DISPATCH(KERNEL_T, ...)                                             \
  switch (U * 2 + (nt ? 1 : 0)) {                                           \
  case 2: KERNEL_T(1, false)<<<blocks, 256, 0, s>>>(__VA_ARGS__); break;    \
  case 3: KERNEL_T(1, true)<<<blocks, 256, 0, s>>>(__VA_ARGS__); break;     \
  case 4: KERNEL_T(2, false)<<<blocks, 256, 0, s>>>(__VA_ARGS__); break;    \
  case 5: KERNEL_T(2, true)<<<blocks, 256, 0, s>>>(__VA_ARGS__); break;     \
  case 8: KERNEL_T(4, false)<<<blocks, 256, 0, s>>>(__VA_ARGS__); break;    \
  case 9: KERNEL_T(4, true)<<<blocks, 256, 0, s>>>(__VA_ARGS__); break;     \
  case 16: KERNEL_T(8, false)<<<blocks, 256, 0, s>>>(__VA_ARGS__); break;   \
  case 17: KERNEL_T(8, true)<<<blocks, 256, 0, s>>>(__VA_ARGS__); break;    \
  default: return -1;                                                       \
  }

#define COPY_T(u, nt) k_copy<u, nt>
#define REG_T(u, nt) k_fixed_reg<false, false, u, nt>

extern "C" int tune_copy(const void *in, void *out, uint64_t nchunks, int U, int nt, int blocks,
                         void *stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  DISPATCH(COPY_T, static_cast<const u32x4 *>(in), static_cast<u32x4 *>(out), nchunks)
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

extern "C" int tune_reg(const void *in, void *out, uint64_t nchunks, uint32_t cpr, const void *prog,
                        int U, int nt, int blocks, void *stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  DISPATCH(REG_T, static_cast<const u32x4 *>(in), static_cast<u32x4 *>(out), nchunks, cpr,
           static_cast<const reg_word *>(prog), nullptr, nullptr)
  return hipGetLastError() == hipSuccess ? 0 : -4;
}
