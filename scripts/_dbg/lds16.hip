#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
// ds_read_u16 at 2-mod-4 addresses, base in a VGPR + immediate offsets
__global__ void k(unsigned* out, int sh) {
  __shared__ uint16_t s[2048];
  for (int i = threadIdx.x; i < 2048; i += 64) s[i] = (uint16_t)i;
  __syncthreads();
  const int base = threadIdx.x + sh;  // element index (odd for odd lanes)
  const char* p = reinterpret_cast<const char*>(s) + base * 2;
  uint16_t a = *reinterpret_cast<const uint16_t*>(p);
  uint16_t b = *reinterpret_cast<const uint16_t*>(p + 116);
  uint16_t c = *reinterpret_cast<const uint16_t*>(p + 462);
  out[threadIdx.x * 3 + 0] = a;
  out[threadIdx.x * 3 + 1] = b;
  out[threadIdx.x * 3 + 2] = c;
}
int main() {
  unsigned* d; hipMalloc(&d, 64 * 3 * 4);
  k<<<1, 64>>>(d, 0);
  unsigned h[192]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int t = 0; t < 64; ++t) {
    if (h[3*t] != (unsigned)t || h[3*t+1] != (unsigned)(t + 58) || h[3*t+2] != (unsigned)(t + 231)) {
      if (bad < 6) printf("lane %d: %u %u %u (want %d %d %d)\n", t, h[3*t], h[3*t+1], h[3*t+2], t, t + 58, t + 231);
      ++bad;
    }
  }
  printf("bad lanes %d\n", bad);
  return 0;
}
