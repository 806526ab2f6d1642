// Round-5 probe: does a VALU write of a data VGPR right after a 128-bit
// buffer / global store (no wait state in between) change the stored data on
// gfx950?  Each variant: every lane stores (a, b, c, d) = (lane, 1000+lane,
// 2000+lane, 3000+lane) as one dwordx4, then the next instruction overwrites
// the first data VGPR with 0xdead0000 | lane.  The host counts lanes whose
// first stored dword is not `lane`.
//   0  buffer_store_dwordx4, SGPR soffset (nonzero), VALU overwrite next
//   1  same with s_nop 0 between
//   2  buffer_store_dwordx4, soffset literal 0, VALU overwrite next
//   3  buffer_store_dwordx4 sc0 nt, SGPR soffset, VALU overwrite next
//   4  global_store_dwordx4, VALU overwrite next
//   5  buffer_store_dwordx2 (64-bit data), SGPR soffset, overwrite next
//   6-9  the test store behind 16 other 128-bit stores of the wave (a busy
//      store path): 6 SGPR soffset, 7 + s_nop 0, 8 sc0 nt, 9 literal 0 + s_nop 0
//   10, 11  the store data fresh from an LDS round trip (k_sweep_tile's wide
//      stores), SGPR soffset, overwrite next; 11 four rows back to back
//   12-15  the overwrite as a VOP3 instruction (12 v_cndmask_b32_e64, 13
//      v_cvt_pk_bf16_f32 after an sc0 nt store, 14 v_add3_u32, 15
//      v_cndmask_b32_e64 after an LDS round trip and an sc0 nt store)
//   16, 17  eight buffer_load_dwordx4 in flight when the store issues (the
//      sweep's tap gathers), SGPR soffset; 17 with s_nop 0 before the overwrite
//   18, 19  64 rows per wave back to back (LDS round trip, sc0 nt store with
//      an SGPR soffset, VOP3 overwrite next; 19 with s_nop 0)
// Build: hipcc --offload-arch=gfx950 -O2 -o probe_store_hazard probe_store_hazard.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void k_probe(uint32_t* out, int variant, int soff_bytes) {
  const int lane = (int)(threadIdx.x & 63), wave = (int)(threadIdx.x >> 6);
  const uint32_t a = (uint32_t)lane, b = 1000u + lane, c = 2000u + lane, d = 3000u + lane;
  const uint32_t x = 0xdead0000u | (uint32_t)lane;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0x7fffffff, 0x00020000);
  const uint32_t voff = (uint32_t)(wave * 64 + lane) * 16u;
  const int soff = soff_bytes;
  uint32_t* gp = out + (size_t)soff_bytes / 4 + (size_t)(wave * 64 + lane) * 4;
  if (variant == 0) {
    asm volatile(
        "v_mov_b32 v10, %0\n\tv_mov_b32 v11, %1\n\tv_mov_b32 v12, %2\n\tv_mov_b32 v13, %3\n\t"
        "s_nop 4\n\t"
        "buffer_store_dwordx4 v[10:13], %4, %5, %6 offen\n\t"
        "v_mov_b32 v10, %7\n\t"
        "s_waitcnt vmcnt(0)"
        :: "v"(a), "v"(b), "v"(c), "v"(d), "v"(voff), "s"(rsrc), "s"(soff), "v"(x)
        : "v10", "v11", "v12", "v13", "memory");
  } else if (variant == 1) {
    asm volatile(
        "v_mov_b32 v10, %0\n\tv_mov_b32 v11, %1\n\tv_mov_b32 v12, %2\n\tv_mov_b32 v13, %3\n\t"
        "s_nop 4\n\t"
        "buffer_store_dwordx4 v[10:13], %4, %5, %6 offen\n\t"
        "s_nop 0\n\t"
        "v_mov_b32 v10, %7\n\t"
        "s_waitcnt vmcnt(0)"
        :: "v"(a), "v"(b), "v"(c), "v"(d), "v"(voff), "s"(rsrc), "s"(soff), "v"(x)
        : "v10", "v11", "v12", "v13", "memory");
  } else if (variant == 2) {
    asm volatile(
        "v_mov_b32 v10, %0\n\tv_mov_b32 v11, %1\n\tv_mov_b32 v12, %2\n\tv_mov_b32 v13, %3\n\t"
        "s_nop 4\n\t"
        "buffer_store_dwordx4 v[10:13], %4, %5, 0 offen\n\t"
        "v_mov_b32 v10, %6\n\t"
        "s_waitcnt vmcnt(0)"
        :: "v"(a), "v"(b), "v"(c), "v"(d), "v"(voff + (uint32_t)soff), "s"(rsrc), "v"(x)
        : "v10", "v11", "v12", "v13", "memory");
  } else if (variant == 3) {
    asm volatile(
        "v_mov_b32 v10, %0\n\tv_mov_b32 v11, %1\n\tv_mov_b32 v12, %2\n\tv_mov_b32 v13, %3\n\t"
        "s_nop 4\n\t"
        "buffer_store_dwordx4 v[10:13], %4, %5, %6 offen sc0 nt\n\t"
        "v_mov_b32 v10, %7\n\t"
        "s_waitcnt vmcnt(0)"
        :: "v"(a), "v"(b), "v"(c), "v"(d), "v"(voff), "s"(rsrc), "s"(soff), "v"(x)
        : "v10", "v11", "v12", "v13", "memory");
  } else if (variant == 4) {
    asm volatile(
        "v_mov_b32 v10, %0\n\tv_mov_b32 v11, %1\n\tv_mov_b32 v12, %2\n\tv_mov_b32 v13, %3\n\t"
        "s_nop 4\n\t"
        "global_store_dwordx4 %4, v[10:13], off\n\t"
        "v_mov_b32 v10, %5\n\t"
        "s_waitcnt vmcnt(0)"
        :: "v"(a), "v"(b), "v"(c), "v"(d), "v"(gp), "v"(x)
        : "v10", "v11", "v12", "v13", "memory");
  } else if (variant >= 6 && variant <= 9) {
    // 6: SGPR soffset, 7: + s_nop 0, 8: sc0 nt SGPR soffset, 9: literal-0 soffset + s_nop 0 -- each behind
    // 16 other 128-bit stores from the same registers' neighbours (a busy store path, as in the sweep)
    const uint32_t fill = voff + 4096u * 16u;
#define PRE16 \
    "buffer_store_dwordx4 v[14:17], %4, %5, %6 offen offset:0\n\t" \
    "buffer_store_dwordx4 v[14:17], %4, %5, %6 offen offset:16\n\t" \
    "buffer_store_dwordx4 v[14:17], %4, %5, %6 offen offset:32\n\t" \
    "buffer_store_dwordx4 v[14:17], %4, %5, %6 offen offset:48\n\t" \
    "buffer_store_dwordx4 v[14:17], %4, %5, %6 offen offset:64\n\t" \
    "buffer_store_dwordx4 v[14:17], %4, %5, %6 offen offset:80\n\t" \
    "buffer_store_dwordx4 v[14:17], %4, %5, %6 offen offset:96\n\t" \
    "buffer_store_dwordx4 v[14:17], %4, %5, %6 offen offset:112\n\t" \
    "buffer_store_dwordx4 v[14:17], %4, %5, %6 offen offset:128\n\t" \
    "buffer_store_dwordx4 v[14:17], %4, %5, %6 offen offset:144\n\t" \
    "buffer_store_dwordx4 v[14:17], %4, %5, %6 offen offset:160\n\t" \
    "buffer_store_dwordx4 v[14:17], %4, %5, %6 offen offset:176\n\t" \
    "buffer_store_dwordx4 v[14:17], %4, %5, %6 offen offset:192\n\t" \
    "buffer_store_dwordx4 v[14:17], %4, %5, %6 offen offset:208\n\t" \
    "buffer_store_dwordx4 v[14:17], %4, %5, %6 offen offset:224\n\t" \
    "buffer_store_dwordx4 v[14:17], %4, %5, %6 offen offset:240\n\t"
#define SETUP "v_mov_b32 v10, %0\n\tv_mov_b32 v11, %1\n\tv_mov_b32 v12, %2\n\tv_mov_b32 v13, %3\n\t" \
    "v_mov_b32 v14, %7\n\tv_mov_b32 v15, %7\n\tv_mov_b32 v16, %7\n\tv_mov_b32 v17, %7\n\ts_nop 4\n\t"
    if (variant == 6)
      asm volatile(SETUP PRE16 "buffer_store_dwordx4 v[10:13], %8, %5, %6 offen\n\tv_mov_b32 v10, %7\n\ts_waitcnt vmcnt(0)"
                   :: "v"(a), "v"(b), "v"(c), "v"(d), "v"(fill), "s"(rsrc), "s"(soff), "v"(x), "v"(voff)
                   : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "memory");
    else if (variant == 7)
      asm volatile(SETUP PRE16 "buffer_store_dwordx4 v[10:13], %8, %5, %6 offen\n\ts_nop 0\n\tv_mov_b32 v10, %7\n\ts_waitcnt vmcnt(0)"
                   :: "v"(a), "v"(b), "v"(c), "v"(d), "v"(fill), "s"(rsrc), "s"(soff), "v"(x), "v"(voff)
                   : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "memory");
    else if (variant == 8)
      asm volatile(SETUP PRE16 "buffer_store_dwordx4 v[10:13], %8, %5, %6 offen sc0 nt\n\tv_mov_b32 v10, %7\n\ts_waitcnt vmcnt(0)"
                   :: "v"(a), "v"(b), "v"(c), "v"(d), "v"(fill), "s"(rsrc), "s"(soff), "v"(x), "v"(voff)
                   : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "memory");
    else
      asm volatile(SETUP PRE16 "buffer_store_dwordx4 v[10:13], %8, %5, 0 offen\n\ts_nop 0\n\tv_mov_b32 v10, %7\n\ts_waitcnt vmcnt(0)"
                   :: "v"(a), "v"(b), "v"(c), "v"(d), "v"(fill), "s"(rsrc), "s"(soff), "v"(x), "v"(voff + (uint32_t)soff)
                   : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "memory");
#undef PRE16
#undef SETUP
  } else if (variant == 10 || variant == 11) {
    // 10: the store data straight from an LDS round trip (ds_write_b128,
    // s_waitcnt, ds_read_b128, s_waitcnt) as in k_sweep_tile's wide stores,
    // SGPR soffset, VALU overwrite next; 11: the same with 4 such rows per
    // wave back to back (the sweep's flush loop)
    __shared__ __attribute__((aligned(16))) uint32_t lds[256 * 4];
    const uint32_t la = (uint32_t)(uintptr_t)&lds[threadIdx.x * 4];
    const int reps = variant == 10 ? 1 : 4;
    for (int r = 0; r < reps; ++r) {
      asm volatile(
          "v_mov_b32 v10, %0\n\tv_mov_b32 v11, %1\n\tv_mov_b32 v12, %2\n\tv_mov_b32 v13, %3\n\t"
          "ds_write_b128 %8, v[10:13]\n\t"
          "v_mov_b32 v10, 0\n\tv_mov_b32 v11, 0\n\tv_mov_b32 v12, 0\n\tv_mov_b32 v13, 0\n\t"
          "s_waitcnt lgkmcnt(0)\n\t"
          "ds_read_b128 v[10:13], %8\n\t"
          "s_waitcnt lgkmcnt(0)\n\t"
          "buffer_store_dwordx4 v[10:13], %4, %5, %6 offen\n\t"
          "v_mov_b32 v10, %7\n\t"
          "s_waitcnt lgkmcnt(0)"
          :: "v"(a), "v"(b), "v"(c), "v"(d), "v"(voff + (uint32_t)r * 0u), "s"(rsrc), "s"(soff), "v"(x), "v"(la)
          : "v10", "v11", "v12", "v13", "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else if (variant >= 12 && variant <= 15) {
    // the overwrite as a VOP3 instruction (k_sweep_tile's flagged pairs):
    // 12 v_cndmask_b32_e64, 13 v_cvt_pk_bf16_f32 (sc0 nt store), 14 v_add3_u32,
    // 15 v_cndmask_b32_e64 after an LDS round trip (sc0 nt store); SGPR soffset
    __shared__ __attribute__((aligned(16))) uint32_t lds2[256 * 4];
    const uint32_t la = (uint32_t)(uintptr_t)&lds2[threadIdx.x * 4];
    const float fx = (float)lane;
    if (variant == 12)
      asm volatile(
          "v_mov_b32 v10, %0\n\tv_mov_b32 v11, %1\n\tv_mov_b32 v12, %2\n\tv_mov_b32 v13, %3\n\t"
          "v_cmp_eq_u32_e64 s[40:41], 1, %8\n\ts_nop 4\n\t"
          "buffer_store_dwordx4 v[10:13], %4, %5, %6 offen\n\t"
          "v_cndmask_b32_e64 v10, %7, %7, s[40:41]\n\t"
          "s_waitcnt vmcnt(0)"
          :: "v"(a), "v"(b), "v"(c), "v"(d), "v"(voff), "s"(rsrc), "s"(soff), "v"(x), "v"(lane & 1)
          : "v10", "v11", "v12", "v13", "s40", "s41", "memory");
    else if (variant == 13)
      asm volatile(
          "v_mov_b32 v10, %0\n\tv_mov_b32 v11, %1\n\tv_mov_b32 v12, %2\n\tv_mov_b32 v13, %3\n\ts_nop 4\n\t"
          "buffer_store_dwordx4 v[10:13], %4, %5, %6 offen sc0 nt\n\t"
          "v_cvt_pk_bf16_f32 v10, %7, 0\n\t"
          "s_waitcnt vmcnt(0)"
          :: "v"(a), "v"(b), "v"(c), "v"(d), "v"(voff), "s"(rsrc), "s"(soff), "v"(fx)
          : "v10", "v11", "v12", "v13", "memory");
    else if (variant == 14)
      asm volatile(
          "v_mov_b32 v10, %0\n\tv_mov_b32 v11, %1\n\tv_mov_b32 v12, %2\n\tv_mov_b32 v13, %3\n\ts_nop 4\n\t"
          "buffer_store_dwordx4 v[10:13], %4, %5, %6 offen\n\t"
          "v_add3_u32 v10, %7, %7, %7\n\t"
          "s_waitcnt vmcnt(0)"
          :: "v"(a), "v"(b), "v"(c), "v"(d), "v"(voff), "s"(rsrc), "s"(soff), "v"(x)
          : "v10", "v11", "v12", "v13", "memory");
    else
      asm volatile(
          "v_mov_b32 v10, %0\n\tv_mov_b32 v11, %1\n\tv_mov_b32 v12, %2\n\tv_mov_b32 v13, %3\n\t"
          "v_cmp_eq_u32_e64 s[40:41], 1, %8\n\t"
          "ds_write_b128 %9, v[10:13]\n\t"
          "v_mov_b32 v10, 0\n\tv_mov_b32 v11, 0\n\tv_mov_b32 v12, 0\n\tv_mov_b32 v13, 0\n\t"
          "s_waitcnt lgkmcnt(0)\n\t"
          "ds_read_b128 v[10:13], %9\n\t"
          "s_waitcnt lgkmcnt(0)\n\t"
          "buffer_store_dwordx4 v[10:13], %4, %5, %6 offen sc0 nt\n\t"
          "v_cndmask_b32_e64 v10, %7, %7, s[40:41]\n\t"
          "s_waitcnt vmcnt(0)"
          :: "v"(a), "v"(b), "v"(c), "v"(d), "v"(voff), "s"(rsrc), "s"(soff), "v"(x), "v"(lane & 1), "v"(la)
          : "v10", "v11", "v12", "v13", "s40", "s41", "memory");
  } else if (variant == 16 || variant == 17) {
    // the texture path busy: 8 buffer_load_dwordx4 of the wave in flight (the
    // sweep's tap gathers) when the store issues; SGPR soffset, sc0 nt store,
    // v_cndmask_b32_e64 overwrite next (17: with s_nop 0 between)
    const uint32_t lo = (uint32_t)(wave * 64 + lane) * 16u + 4096u * 16u;
    if (variant == 16)
      asm volatile(
          "v_mov_b32 v10, %0\n\tv_mov_b32 v11, %1\n\tv_mov_b32 v12, %2\n\tv_mov_b32 v13, %3\n\t"
          "v_cmp_eq_u32_e64 s[40:41], 1, %8\n\ts_nop 4\n\t"
          "buffer_load_dwordx4 v[20:23], %9, %5, 0 offen\n\t"
          "buffer_load_dwordx4 v[24:27], %9, %5, 0 offen offset:16\n\t"
          "buffer_load_dwordx4 v[28:31], %9, %5, 0 offen offset:32\n\t"
          "buffer_load_dwordx4 v[32:35], %9, %5, 0 offen offset:48\n\t"
          "buffer_load_dwordx4 v[36:39], %9, %5, 0 offen offset:64\n\t"
          "buffer_load_dwordx4 v[40:43], %9, %5, 0 offen offset:80\n\t"
          "buffer_load_dwordx4 v[44:47], %9, %5, 0 offen offset:96\n\t"
          "buffer_load_dwordx4 v[48:51], %9, %5, 0 offen offset:112\n\t"
          "buffer_store_dwordx4 v[10:13], %4, %5, %6 offen sc0 nt\n\t"
          "v_cndmask_b32_e64 v10, %7, %7, s[40:41]\n\t"
          "s_waitcnt vmcnt(0)"
          :: "v"(a), "v"(b), "v"(c), "v"(d), "v"(voff), "s"(rsrc), "s"(soff), "v"(x), "v"(lane & 1), "v"(lo)
          : "v10", "v11", "v12", "v13", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30",
            "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45",
            "v46", "v47", "v48", "v49", "v50", "v51", "s40", "s41", "memory");
    else
      asm volatile(
          "v_mov_b32 v10, %0\n\tv_mov_b32 v11, %1\n\tv_mov_b32 v12, %2\n\tv_mov_b32 v13, %3\n\t"
          "v_cmp_eq_u32_e64 s[40:41], 1, %8\n\ts_nop 4\n\t"
          "buffer_load_dwordx4 v[20:23], %9, %5, 0 offen\n\t"
          "buffer_load_dwordx4 v[24:27], %9, %5, 0 offen offset:16\n\t"
          "buffer_load_dwordx4 v[28:31], %9, %5, 0 offen offset:32\n\t"
          "buffer_load_dwordx4 v[32:35], %9, %5, 0 offen offset:48\n\t"
          "buffer_load_dwordx4 v[36:39], %9, %5, 0 offen offset:64\n\t"
          "buffer_load_dwordx4 v[40:43], %9, %5, 0 offen offset:80\n\t"
          "buffer_load_dwordx4 v[44:47], %9, %5, 0 offen offset:96\n\t"
          "buffer_load_dwordx4 v[48:51], %9, %5, 0 offen offset:112\n\t"
          "buffer_store_dwordx4 v[10:13], %4, %5, %6 offen sc0 nt\n\t"
          "s_nop 0\n\t"
          "v_cndmask_b32_e64 v10, %7, %7, s[40:41]\n\t"
          "s_waitcnt vmcnt(0)"
          :: "v"(a), "v"(b), "v"(c), "v"(d), "v"(voff), "s"(rsrc), "s"(soff), "v"(x), "v"(lane & 1), "v"(lo)
          : "v10", "v11", "v12", "v13", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30",
            "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45",
            "v46", "v47", "v48", "v49", "v50", "v51", "s40", "s41", "memory");
  } else if (variant == 18 || variant == 19) {
    // sustained store traffic as in the sweep: 64 rows per wave, each an LDS
    // round trip, a 128-bit sc0 nt store with the row's SGPR soffset, and a
    // VOP3 overwrite of the first data VGPR right after (19: s_nop 0 between);
    // only the last row's first dword is checked (the earlier rows land past
    // the checked words)
    __shared__ __attribute__((aligned(16))) uint32_t lds3[256 * 4];
    const uint32_t la = (uint32_t)(uintptr_t)&lds3[threadIdx.x * 4];
    for (int r = 63; r >= 0; --r) {
      const int so = soff + r * 65536;
      if (variant == 18)
        asm volatile(
            "v_mov_b32 v10, %0\n\tv_mov_b32 v11, %1\n\tv_mov_b32 v12, %2\n\tv_mov_b32 v13, %3\n\t"
            "v_cmp_eq_u32_e64 s[40:41], 1, %8\n\t"
            "ds_write_b128 %9, v[10:13]\n\t"
            "s_waitcnt lgkmcnt(0)\n\t"
            "ds_read_b128 v[10:13], %9\n\t"
            "s_waitcnt lgkmcnt(0)\n\t"
            "buffer_store_dwordx4 v[10:13], %4, %5, %6 offen sc0 nt\n\t"
            "v_cndmask_b32_e64 v10, %7, %7, s[40:41]"
            :: "v"(a), "v"(b), "v"(c), "v"(d), "v"(voff), "s"(rsrc), "s"(so), "v"(x), "v"(lane & 1), "v"(la)
            : "v10", "v11", "v12", "v13", "s40", "s41", "memory");
      else
        asm volatile(
            "v_mov_b32 v10, %0\n\tv_mov_b32 v11, %1\n\tv_mov_b32 v12, %2\n\tv_mov_b32 v13, %3\n\t"
            "v_cmp_eq_u32_e64 s[40:41], 1, %8\n\t"
            "ds_write_b128 %9, v[10:13]\n\t"
            "s_waitcnt lgkmcnt(0)\n\t"
            "ds_read_b128 v[10:13], %9\n\t"
            "s_waitcnt lgkmcnt(0)\n\t"
            "buffer_store_dwordx4 v[10:13], %4, %5, %6 offen sc0 nt\n\t"
            "s_nop 0\n\t"
            "v_cndmask_b32_e64 v10, %7, %7, s[40:41]"
            :: "v"(a), "v"(b), "v"(c), "v"(d), "v"(voff), "s"(rsrc), "s"(so), "v"(x), "v"(lane & 1), "v"(la)
            : "v10", "v11", "v12", "v13", "s40", "s41", "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else if (variant == 5) {
    asm volatile(
        "v_mov_b32 v10, %0\n\tv_mov_b32 v11, %1\n\tv_mov_b32 v12, %2\n\tv_mov_b32 v13, %3\n\t"
        "s_nop 4\n\t"
        "buffer_store_dwordx2 v[10:11], %4, %5, %6 offen\n\t"
        "v_mov_b32 v10, %7\n\t"
        "s_waitcnt vmcnt(0)"
        :: "v"(a), "v"(b), "v"(c), "v"(d), "v"(voff), "s"(rsrc), "s"(soff), "v"(x)
        : "v10", "v11", "v12", "v13", "memory");
  }
}

int main() {
  const int threads = 256, blocks = 1024, soff = 64;
  const size_t n = (size_t)threads * 4 + soff / 4 + (size_t)4096 * 4 + 1024 + (size_t)64 * 65536 / 4;
  uint32_t* d = nullptr;
  if (hipMalloc(&d, n * 4) != hipSuccess) return 2;
  std::vector<uint32_t> h(n);
  for (int v = 0; v <= 19; ++v) {
    long bad = 0, runs = 0;
    for (int rep = 0; rep < 20; ++rep) {
      hipMemset(d, 0, n * 4);
      // every block writes the same words (same values), so the result is the
      // last writer's: run many blocks so the store path is busy
      hipLaunchKernelGGL(k_probe, dim3(blocks), dim3(threads), 0, 0, d, v, soff);
      if (hipDeviceSynchronize() != hipSuccess) { printf("variant %d: launch failed\n", v); return 3; }
      hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
      for (int t = 0; t < threads; ++t) {
        const uint32_t got = h[soff / 4 + (size_t)t * 4];
        bad += got != (uint32_t)(t & 63);
        ++runs;
      }
    }
    // which lanes of a wave (last repetition)
    unsigned long long lanes = 0ull;
    for (int t = 0; t < threads; ++t)
      if (h[soff / 4 + (size_t)t * 4] != (uint32_t)(t & 63)) lanes |= 1ull << (t & 63);
    printf("variant %d: %ld of %ld lanes stored a wrong first dword (lanes mask %016llx)\n", v, bad, runs, lanes);
  }
  hipFree(d);
  return 0;
}
