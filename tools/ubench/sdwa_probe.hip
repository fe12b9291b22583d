// Probe (dev tool): does v_cvt_i32_f32 with SDWA dst_sel:BYTE_n place the low byte of the truncated
// integer into byte n (others preserved)?  Compares against the v_cvt + v_perm packing.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
template <int MODE>
__global__ void k(const float* x, unsigned* y) {
  const int t = threadIdx.x;
  float a = x[4 * t], b = x[4 * t + 1], c = x[4 * t + 2], d = x[4 * t + 3];
  unsigned r = 0;
  // mode 0: four separate statements; 1: one block, back to back (the failing form)
  if (MODE == 0) {
    asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PRESERVE src0_sel:DWORD" : "+v"(r) : "v"(a));
    asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD" : "+v"(r) : "v"(b));
    asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD" : "+v"(r) : "v"(c));
    asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD" : "+v"(r) : "v"(d));
  } else {
    asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD\n\t"
                 "v_cvt_i32_f32_sdwa %0, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD\n\t"
                 "v_cvt_i32_f32_sdwa %0, %3 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD\n\t"
                 "v_cvt_i32_f32_sdwa %0, %4 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD"
                 : "=&v"(r) : "v"(a), "v"(b), "v"(c), "v"(d));
  }
  y[t] = r;
}
int main() {
  const int n = 64 * 64;
  float hx[4 * 4096];
  for (int i = 0; i < 4 * n / 4; ++i) hx[i] = (float)((i * 37) % 255 - 127) + 0.25f * ((i % 4) - 1.5f);
  float* dx; unsigned* dy;
  hipMalloc(&dx, sizeof(hx)); hipMalloc(&dy, n / 4 * 4 * sizeof(unsigned));
  hipMemcpy(dx, hx, sizeof(hx), hipMemcpyHostToDevice);
  for (int mode = 0; mode < 2; ++mode) {
  if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(1024), 0, 0, dx, dy);
  else hipLaunchKernelGGL(k<1>, dim3(1), dim3(1024), 0, 0, dx, dy);
  unsigned hy[1024];
  hipMemcpy(hy, dy, sizeof(hy), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int t = 0; t < 1024; ++t) {
    unsigned e = 0;
    for (int j = 0; j < 4; ++j) e |= ((unsigned)(int)truncf(hx[4 * t + j]) & 0xffu) << (8 * j);
    if (e != hy[t]) { if (bad < 5) printf("t=%d got %08x want %08x\n", t, hy[t], e); ++bad; }
  }
  printf("sdwa byte pack, %s: %s (%d mismatches of 1024)\n", mode ? "one block, back to back" : "separate statements",
         bad ? "DIFFERENT" : "exact", bad);
  }
  return 0;
}
