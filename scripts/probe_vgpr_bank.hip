// Probe: v_fma_f32 issue rate on gfx950 as a function of the VGPR banks of
// its three sources (bank = register index mod 4), 1..8 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o probe_vgpr_bank probe_vgpr_bank.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CLOB "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15", \
             "v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31", \
             "v32","v33","v34","v35","v36","v37","v38","v39"

// 8 independent FMAs per line group; destinations v32..v39 (banks 0..3)
// A: sources in three distinct banks, none equal to each other
#define BODY_A \
  "v_fma_f32 v32, v1, v2, v3\n" "v_fma_f32 v33, v5, v6, v7\n" "v_fma_f32 v34, v9, v10, v11\n" \
  "v_fma_f32 v35, v13, v14, v15\n" "v_fma_f32 v36, v17, v18, v19\n" "v_fma_f32 v37, v21, v22, v23\n" \
  "v_fma_f32 v38, v25, v26, v27\n" "v_fma_f32 v39, v29, v30, v31\n"
// B: all three sources in the same bank
#define BODY_B \
  "v_fma_f32 v32, v0, v4, v8\n" "v_fma_f32 v33, v1, v5, v9\n" "v_fma_f32 v34, v2, v6, v10\n" \
  "v_fma_f32 v35, v3, v7, v11\n" "v_fma_f32 v36, v12, v16, v20\n" "v_fma_f32 v37, v13, v17, v21\n" \
  "v_fma_f32 v38, v14, v18, v22\n" "v_fma_f32 v39, v15, v19, v23\n"
// C: two sources share a bank, third differs
#define BODY_C \
  "v_fma_f32 v32, v0, v4, v1\n" "v_fma_f32 v33, v1, v5, v2\n" "v_fma_f32 v34, v2, v6, v3\n" \
  "v_fma_f32 v35, v3, v7, v0\n" "v_fma_f32 v36, v12, v16, v13\n" "v_fma_f32 v37, v13, v17, v14\n" \
  "v_fma_f32 v38, v14, v18, v15\n" "v_fma_f32 v39, v15, v19, v12\n"
// D: VOP2 fmac (dst is the addend), sources in distinct banks
#define BODY_D \
  "v_fmac_f32 v32, v1, v2\n" "v_fmac_f32 v33, v5, v6\n" "v_fmac_f32 v34, v9, v10\n" "v_fmac_f32 v35, v13, v14\n" \
  "v_fmac_f32 v36, v17, v18\n" "v_fmac_f32 v37, v21, v22\n" "v_fmac_f32 v38, v25, v26\n" "v_fmac_f32 v39, v29, v30\n"

#define KERNEL(name, body) \
__global__ void name(float* out, int iters) { \
  for (int i = 0; i < iters; ++i) { \
    asm volatile(body body body body ::: CLOB); \
  } \
  if (threadIdx.x == 1234567) out[0] = 0.f; \
}
KERNEL(k_a, BODY_A)
KERNEL(k_b, BODY_B)
KERNEL(k_c, BODY_C)
KERNEL(k_d, BODY_D)

int main() {
  float* out;
  hipMalloc(&out, 4);
  int dev = 0; hipDeviceProp_t p; hipGetDeviceProperties(&p, dev);
  const int cus = p.multiProcessorCount;
  const int iters = 20000;
  void (*ks[4])(float*, int) = {k_a, k_b, k_c, k_d};
  const char* names[4] = {"A distinct banks", "B same bank x3", "C two share", "D fmac distinct"};
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int waves = 1; waves <= 8; waves *= 2) {
    for (int v = 0; v < 4; ++v) {
      // one block of 64*4*waves threads per CU -> `waves` waves on each SIMD
      dim3 grid(cus), block(256 * waves > 1024 ? 1024 : 256 * waves);
      int blocks = cus * ((256 * waves) / block.x);
      hipLaunchKernelGGL(ks[v], dim3(blocks), block, 0, 0, out, 100);
      hipDeviceSynchronize();
      hipEventRecord(e0);
      hipLaunchKernelGGL(ks[v], dim3(blocks), block, 0, 0, out, iters);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      const double fma_wave_instr = (double)iters * 32 * blocks * (block.x / 64);
      const double per_simd = fma_wave_instr / (cus * 4);
      printf("waves/SIMD %d  %-18s %8.3f ms  %.3f ns per wave-FMA per SIMD  (%.2f cycles @2.4GHz)\n", waves,
             names[v], ms, ms * 1e6 / per_simd, ms * 1e6 / per_simd * 2.4);
    }
  }
  return 0;
}
