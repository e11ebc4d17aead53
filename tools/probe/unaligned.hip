// Probe: are 16-byte global loads/stores at 1/4-byte-aligned addresses
// correct on this device (SH_MEM_CONFIG unaligned mode), and how fast is a
// per-lane (scattered-record) 16B copy vs a dword copy?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_copy16(const uint8_t* in, uint8_t* out, int n, int sh_in, int sh_out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    u32x4 v = *reinterpret_cast<const u32x4*>(in + sh_in + 16 * i);
    *reinterpret_cast<u32x4*>(out + sh_out + 16 * i) = v;
  }
}
// each lane copies its own "record" of rec bytes (16B steps) from in+lane*rec
__global__ void k_lane16(const uint8_t* in, uint8_t* out, long nrec, int rec, int sh) {
  long r = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (r >= nrec) return;
  const uint8_t* s = in + r * rec + sh;
  uint8_t* d = out + r * rec + 4;
  for (int k = 0; k < rec / 16 - 1; ++k)
    *reinterpret_cast<u32x4*>(d + 16 * k) = *reinterpret_cast<const u32x4*>(s + 16 * k);
}
__global__ void k_lane4(const uint8_t* in, uint8_t* out, long nrec, int rec, int sh) {
  long r = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (r >= nrec) return;
  const uint8_t* s = in + r * rec + (sh & ~3);
  uint8_t* d = out + r * rec + 4;
  for (int k = 0; k < rec / 4 - 4; ++k)
    *reinterpret_cast<uint32_t*>(d + 4 * k) = __builtin_amdgcn_alignbyte(
        *reinterpret_cast<const uint32_t*>(s + 4 * k + 4), *reinterpret_cast<const uint32_t*>(s + 4 * k), sh & 3);
}
int main() {
  const int n = 1 << 20;
  std::vector<uint8_t> h(16 * n + 64);
  for (size_t i = 0; i < h.size(); ++i) h[i] = uint8_t(i * 131 + 7);
  uint8_t *din, *dout;
  hipMalloc(&din, h.size()); hipMalloc(&dout, h.size());
  hipMemcpy(din, h.data(), h.size(), hipMemcpyHostToDevice);
  for (int shi : {0, 1, 2, 3, 4, 8, 12}) for (int sho : {0, 4, 8, 1}) {
    hipMemset(dout, 0, h.size());
    k_copy16<<<n / 256, 256>>>(din, dout, n, shi, sho);
    hipError_t e = hipDeviceSynchronize();
    std::vector<uint8_t> o(h.size());
    hipMemcpy(o.data(), dout, o.size(), hipMemcpyDeviceToHost);
    bool ok = e == hipSuccess && !memcmp(o.data() + sho, h.data() + shi, 16 * (size_t)n);
    printf("copy16 in+%d out+%d: %s\n", shi, sho, ok ? "ok" : (e == hipSuccess ? "WRONG" : hipGetErrorString(e)));
  }
  // scattered per-lane 16B vs 4B copies: 1M records of 192 bytes
  const long nrec = 1 << 20; const int rec = 192;
  uint8_t *a, *b; hipMalloc(&a, nrec * rec + 64); hipMalloc(&b, nrec * rec + 64);
  hipMemset(a, 1, nrec * rec + 64);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int sh : {0, 1, 4}) {
    for (int variant = 0; variant < 2; ++variant) {
      for (int w = 0; w < 3; ++w) {
        if (variant == 0) k_lane16<<<nrec / 256, 256>>>(a, b, nrec, rec, sh);
        else k_lane4<<<nrec / 256, 256>>>(a, b, nrec, rec, sh);
      }
      hipEventRecord(e0);
      for (int w = 0; w < 10; ++w) {
        if (variant == 0) k_lane16<<<nrec / 256, 256>>>(a, b, nrec, rec, sh);
        else k_lane4<<<nrec / 256, 256>>>(a, b, nrec, rec, sh);
      }
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 10;
      double bytes = 2.0 * nrec * (rec - 16);
      printf("lane%s sh=%d: %.3f ms  %.0f GB/s\n", variant ? "4 " : "16", sh, ms, bytes / ms / 1e6);
    }
  }
  return 0;
}
