// Development probe: print the lane mapping of v_permlane16_swap_b32 / v_permlane32_swap_b32.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* o) {
  int x = threadIdx.x, y = 100 + threadIdx.x;
  int a = x, b = y;
  asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  o[threadIdx.x] = a;
  o[64 + threadIdx.x] = b;
  a = x, b = y;
  asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  o[128 + threadIdx.x] = a;
  o[192 + threadIdx.x] = b;
}
int main() {
  int* d;
  hipMalloc(&d, 256 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  int h[256];
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  const char* nm[] = {"p32 vdst", "p32 vsrc", "p16 vdst", "p16 vsrc"};
  for (int r = 0; r < 4; ++r) {
    printf("%s:", nm[r]);
    for (int i = 0; i < 64; ++i) printf(" %d", h[r * 64 + i]);
    printf("\n");
  }
}
