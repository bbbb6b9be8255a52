// Where do the blocks of a persistent 2-blocks-per-CU grid land?  Launches G blocks of 256
// threads holding ~73 KB of LDS each (the GEMM's footprint) and records (XCC, SE, CU) per
// block from the hardware-id registers, plus a per-block spin so all blocks are co-resident.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ __launch_bounds__(256, 2) void where(int* out, int spin) {
  __shared__ float pad[18 * 1024];
  if (threadIdx.x == 0) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    out[blockIdx.x * 4 + 0] = xcc & 0xf;
    out[blockIdx.x * 4 + 1] = (hw >> 13) & 0x7;     // SE_ID
    out[blockIdx.x * 4 + 2] = (hw >> 8) & 0xf;      // CU_ID
    out[blockIdx.x * 4 + 3] = (hw >> 12) & 0x1;     // SH_ID
  }
  float s = 0.f;
  for (int i = 0; i < spin; ++i) s += pad[(threadIdx.x + i) & 1023];
  if (s == 1234.f) out[0] = -1;
}

int main(int argc, char** argv) {
  const int G = argc > 1 ? atoi(argv[1]) : 512;
  int* d;
  hipMalloc(&d, G * 4 * sizeof(int));
  hipLaunchKernelGGL(where, dim3(G), dim3(256), 0, 0, d, 200000);
  hipDeviceSynchronize();
  int* h = (int*)malloc(G * 4 * sizeof(int));
  hipMemcpy(h, d, G * 4 * sizeof(int), hipMemcpyDeviceToHost);
  for (int b = 0; b < G; ++b) printf("%d %d %d %d %d\n", b, h[4 * b], h[4 * b + 1], h[4 * b + 3], h[4 * b + 2]);
  return 0;
}
