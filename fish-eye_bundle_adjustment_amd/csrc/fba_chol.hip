// fba_chol.hip -- fp64 sparse (block) Cholesky of the reduced camera system on gfx950 (MI355X).
//
// The reference inverts the bordered normal matrix explicitly, Cx = [N G; G' 0]^-1
// (main.m:428-440).  Here the tie points have already been eliminated (Schur complement), the
// images are in nested-dissection order (fba_order.cpp), so the image-image part of the reduced
// system S is block sparse, and the border is folded in LOCALLY as M = S + A A' with A = G_l W^1/2
// restricted to the first n_loc image slots (SPD whenever the bordered matrix is nonsingular and
// those images fix the datum; W = one equilibrating weight per constraint column, fba_kernels.hip
// k_border_weights) -- so M keeps the sparsity of S, and
//
//   M = L L'        right-looking block Cholesky, NB = 128, one batched step per level of the
//                   elimination tree (the columns of a level are independent):
//     k_potrf128    the level's 128x128 diagonal blocks, one LDS-resident workgroup each: 8
//                   sub-panels of 16 (16x16 factor in registers with DPP broadcasts, its 16x16
//                   inverse, then the in-block panel solve and trailing update on
//                   v_mfma_f64_16x16x4_f64); writes L_kk and the eight 16x16 inverses D_s = L_ss^-1
//     k_trsm128     the panel blocks of those columns, X = A L_kk^-T by blocked substitution
//                   X_s = (A_s - sum_{t<s} X_t L_st^T) D_s^T: all MFMA, 16 rows per wave
//     k_syrk_multi  the trailing updates of the level, C -= sum_k X_ik X_jk^T, 64x64 quarters, K = 128
//                   per source column staged through LDS in 32-deep slices; targets with many sources
//                   split into groups (scratch quarters; the last group to arrive adds them in order)
//   forward solve   the right-hand sides [r | A | B] (B = G D, D an equilibration over all images)
//                   are stored as extra ROWS below M (one extra block row, in every panel), so the
//                   panel solves compute Y' = (L^-1 [r A B])' as a by-product
//   border combine  the 14x14 system of k_border_combine restores the exact bordered solution:
//                   u = y + A~ z + B~ k with z = A~'u and B~'u = 0
//   backward solve  L' x = u with the 128x128 diagonal-block inverses (k_trtri128, all blocks in
//                   parallel), then one launch per level, top down (k_bwd_wave)
// so delta_c = -x satisfies [S G; G' 0][delta; lambda] = [-r; 0] as the reference's bordered
// system does.
#include "fba_internal.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <utility>

namespace fba {

typedef double dbl4 __attribute__((ext_vector_type(4)));

constexpr int CB = 128;   // outer block
constexpr int IB = 16;    // inner block (MFMA tile)
constexpr int LDA = 130;  // LDS row stride in doubles for 128-wide tiles: bank = (4r + 2k) mod 64

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {  // a DPP-permuted copy of v (all rows, all banks)
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

// In-launch hand-off of a factored diagonal block (k_panel): the potrf workgroup stores L_kk and its
// leaf inverses WRITE-THROUGH (sc1, buffer stores on a descriptor based at the block), drains its
// stores in every wave, and one lane sets the column's flag with an agent-scope atomic; the panel
// workgroups poll that flag relaxed and read the payload with sc1 loads (no stale L1/L2 copies on any
// XCD).  Flags are zeroed by a memset node ahead of the factorisation (one epoch per launch).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
constexpr int SC1 = 16;  // buffer aux bits: sc1 (write-through / L1 bypass)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t block_rsrc(const void* base, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t r, int64_t off_bytes, double2 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)off_bytes, 0, SC1);
}
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t r, int64_t off_bytes, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, (int)off_bytes, 0, SC1);
}
__device__ __forceinline__ double2 ld_sc1(__amdgpu_buffer_rsrc_t r, int64_t off_bytes) {
    return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off_bytes, 0, SC1));
}
// Bounded polls.  Every wait in this file gives up after scal[SCAL_SPINS] sleeps (the context's bound:
// default 1 << 22, ~0.3 s; FBA_FLAG_SPINS at context creation lowers it, to force the path in a test) and then
// RAISES THE ABORT: scal[1] = -1.0 (agent-scope store).  Every other poll checks the abort word every 64
// sleeps (not on its first miss: that load would sit on every hand-off's critical path) and stops too, so
// after one expiry the whole launch drains within about a millisecond; a k_chol_flow record that has not started yet is skipped entirely, k_bwd_flow's
// workgroups return at once, and k_update leaves xhat untouched (fba_kernels.hip): the step fails with
// FBA_ERR_HIP and xhat is as before it.  The sync words are zeroed again ahead of the next factorisation
// (k_border_rhs), so a later step runs normally.
__device__ __forceinline__ bool hand_off_aborted(const double* scal) {  // the timeout mark, sign bit of -1.0
    return (long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(scal + 1), __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT) < 0;
}
__device__ __forceinline__ void hand_off_abort(double* scal) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(scal + 1), __builtin_bit_cast(unsigned long long, -1.0),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a non-positive pivot in the block at row k0: the first one is reported (scal[1] = k0 + 1) unless a
// hand-off already aborted (a compare-and-swap from 0, so it never overwrites the abort mark)
__device__ __forceinline__ void pivot_failed(double* scal, int64_t k0) {
    unsigned long long zero = 0ull;
    __hip_atomic_compare_exchange_strong(reinterpret_cast<unsigned long long*>(scal + 1), &zero,
                                         __builtin_bit_cast(unsigned long long, (double)(k0 + 1)), __ATOMIC_RELAXED,
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one missed poll: true when this wait must stop (its own bound reached, or another wait aborted)
__device__ __forceinline__ bool spin_expired(unsigned& spins, double* scal) {
    ++spins;
    if (spins >= (unsigned)scal[SCAL_SPINS] || ((spins & 63u) == 0u && hand_off_aborted(scal))) {
        hand_off_abort(scal);
        return true;
    }
    return false;
}

// 1/sqrt(d) from v_rsq_f64 refined by two Newton steps (full double precision), no IEEE divide
__device__ __forceinline__ double rsqrt_d(double d) {
    double r = __builtin_amdgcn_rsq(d);
    r = r * (1.5 - 0.5 * d * r * r);
    r = r * (1.5 - 0.5 * d * r * r);
    return r;
}

__device__ __forceinline__ dbl4 mfma(double a, double b, dbl4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

template <int L>
__device__ __forceinline__ double bc16(double v) {
    return __builtin_amdgcn_mov_dpp(v, 0x150 + L, 0xF, 0xF, true);
}

// lane index known after unrolling: resolved at compile time
__device__ __forceinline__ double bcl(double v, int l) {
    switch (l) {
        case 0: return bc16<0>(v);
        case 1: return bc16<1>(v);
        case 2: return bc16<2>(v);
        case 3: return bc16<3>(v);
        case 4: return bc16<4>(v);
        case 5: return bc16<5>(v);
        case 6: return bc16<6>(v);
        case 7: return bc16<7>(v);
        case 8: return bc16<8>(v);
        case 9: return bc16<9>(v);
        case 10: return bc16<10>(v);
        case 11: return bc16<11>(v);
        case 12: return bc16<12>(v);
        case 13: return bc16<13>(v);
        case 14: return bc16<14>(v);
        case 15: return bc16<15>(v);
        default: return v;
    }
}

// d += s[lane l of this row] * m, one v_fmac_f64_dpp (row_newbcast:l); l known after unrolling.
// The first use of a freshly written s carries the 2-wait-state VALU-write -> DPP-read gap itself
// (inline asm is opaque to the compiler's hazard recognizer).
__device__ __forceinline__ void fmac_bc_first(double& d, double s, double m, int l) {
    switch (l) {
        case 1: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 2: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:2 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 3: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 4: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:4 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 5: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:5 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 6: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:6 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 7: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:7 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 8: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:8 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 9: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:9 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 10: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:10 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 11: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:11 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 12: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:12 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 13: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:13 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 14: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:14 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 15: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:15 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        default: break;
    }
}
__device__ __forceinline__ void fmac_bc(double& d, double s, double m, int l) {
    switch (l) {
        case 1: asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 2: asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:2 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 3: asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 4: asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:4 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 5: asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:5 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 6: asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:6 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 7: asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:7 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 8: asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:8 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 9: asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:9 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 10: asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:10 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 11: asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:11 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 12: asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:12 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 13: asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:13 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 14: asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:14 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 15: asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:15 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        default: break;
    }
}

// d += s[lane l of this row] * (-m), one v_fmac_f64_dpp with a negated src1 (row_newbcast:l)
__device__ __forceinline__ void fmac_bcn_first(double& d, double s, double m, int l) {
    switch (l) {
        case 1: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, -%2 row_newbcast:1 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 2: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, -%2 row_newbcast:2 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 3: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, -%2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 4: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, -%2 row_newbcast:4 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 5: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, -%2 row_newbcast:5 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 6: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, -%2 row_newbcast:6 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 7: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, -%2 row_newbcast:7 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 8: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, -%2 row_newbcast:8 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 9: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, -%2 row_newbcast:9 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 10: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, -%2 row_newbcast:10 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 11: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, -%2 row_newbcast:11 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 12: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, -%2 row_newbcast:12 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 13: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, -%2 row_newbcast:13 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 14: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, -%2 row_newbcast:14 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 15: asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, -%2 row_newbcast:15 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        default: break;
    }
}
__device__ __forceinline__ void fmac_bcn(double& d, double s, double m, int l) {
    switch (l) {
        case 1: asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:1 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 2: asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:2 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 3: asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 4: asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:4 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 5: asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:5 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 6: asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:6 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 7: asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:7 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 8: asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:8 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 9: asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:9 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 10: asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:10 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 11: asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:11 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 12: asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:12 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 13: asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:13 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 14: asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:14 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        case 15: asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:15 row_mask:0xf bank_mask:0xf" : "+v"(d) : "v"(s), "v"(m)); break;
        default: break;
    }
}

// a fold over a compile-time index sequence (every index a constant expression in the body)
template <int... Q, class F>
__device__ __forceinline__ void bulk_for(std::integer_sequence<int, Q...>, F&& f) {
    (f(std::integral_constant<int, Q>{}), ...);
}

// lane i (< 16) of a wave holds row i of a 16x16 SPD block in a[]; on return a[] holds row i of L
// (lower part) and x[] COLUMN i of L^-1 (x[r] = (L^-1)[r][i]).  Every broadcast L[l][j] feeds both
// the rank-1 update of the factor and the forward substitution of the inverse's columns, each as
// one v_fmac_f64_dpp (negated src1: no separate negation).  The pivot chain per column is
// broadcast -> v_rsq_f64 -> one third-order correction folded into L[i][j] -> the next column's
// update: rsq is good to 2^-24 (measured), so e = d r^2 - 1 and r (1 - e/2 + 3e^2/8) is accurate to
// rounding (max rel. error 2.7e-16 measured, vs 3.0e-16 for two Newton steps).  The pivot test is
// off the chain: a non-positive pivot propagates NaN and is reported (returns false).
// put(j): called once column j of L (a[j] on lanes >= j) and row j of L^-1 (x[j]) are final.
// Issue-bound: ~400 f64 VALU instructions at ~5.6 shader clocks each on one wave (a dependent f64 fma
// is 8.6 clocks, an independent one 5.7: scripts/ubench/leaf_lat.hip); a software-pipelined order that
// spreads each column's updates over the next pivot chain's steps measured slower.
template <class PUT>
__device__ __forceinline__ bool leaf_factor(double (&a)[IB], double (&x)[IB], int lane16, PUT&& put) {
    bool ok = true;
#pragma unroll
    for (int r = 0; r < IB; ++r) x[r] = (r == lane16) ? 1.0 : 0.0;
#pragma unroll
    for (int j = 0; j < IB; ++j) {
        const double d = bcl(a[j], j);
        ok &= d > 0.0;
        const double r = __builtin_amdgcn_rsq(d);
        const double ar = a[j] * r;
        const double t = d * r;
        const double e = __builtin_fma(t, r, -1.0);
        const double p = __builtin_fma(e, 0.375, -0.5);
        const double inv = __builtin_fma(r * e, p, r);
        a[j] = __builtin_fma(ar * e, p, ar);  // lane j: sqrt(d); lanes > j: L[i][j]; lanes < j: unused
        x[j] *= inv;                          // (L^-1)[j][c] final
#pragma unroll
        for (int l = j + 1; l < IB; ++l) {
            if (l == j + 1) fmac_bcn_first(a[l], a[j], a[j], l);  // a[l] -= L[i][j] L[l][j]
            else fmac_bcn(a[l], a[j], a[j], l);
        }
#pragma unroll
        for (int l = j + 1; l < IB; ++l) fmac_bcn(x[l], a[j], x[j], l);  // x[l] -= L[l][j] x[j]
        put(j);
    }
    return ok;
}

__device__ __forceinline__ bool leaf_factor(double (&a)[IB], double (&x)[IB], int lane16) {
    return leaf_factor(a, x, lane16, [](int) {});
}

// ------------------------------------------------------------------------------------------------
// k_potrf128: factor the 128x128 diagonal block at (k0, k0); 512 threads.
// Eight 16-column leaves.  A leaf is factored in registers by wave 0 (lane i = row i) with
// row_newbcast DPP broadcasts: every broadcast L[l][j] feeds both the rank-1 update of the
// leaf and the forward substitution of its inverse D_s = L_ss^-1 (lane c = column c), so the leaf
// factor and its inverse cost one pass.  In-block lookahead: after the panel solve of leaf s, wave 0
// updates the next diagonal tile and factors leaf s+1 while waves 1-3 apply the rest of the update.
// ------------------------------------------------------------------------------------------------

constexpr int POTRF_NT = (CB / IB) * (CB / IB + 1) / 2;  // 36 lower tiles
constexpr int POTRF_THREADS = 512;                          // wave 0: the leaf chain; waves 1-7: the bulk
constexpr int POTRF_NW = POTRF_THREADS / 64;
constexpr size_t POTRF_LDS = sizeof(double) * (POTRF_NT + CB / IB) * IB * 17 + 32 * sizeof(int);  // + the eight D_s, counters

// TS: shader-clock stamps of wave 0's critical path into ts[] (calibration builds only,
// scripts/ubench/chol_ubench.hip)
// potrf_body: factor the 128x128 diagonal block of column col (512 threads); flag != nullptr: publish
// it (k_panel hand-off)
// wait until every flag of a list is set (merged launch: the previous level's updates of this
// workgroup's blocks); one lane polls, bounded, then the whole workgroup
__device__ __forceinline__ void wait_list(const int32_t* __restrict__ wl, int n, unsigned* __restrict__ tflags,
                                          double* __restrict__ scal) {
    if (n <= 0) return;
    if (threadIdx.x == 0)
        for (int q = 0; q < n; ++q) {
            unsigned spins = 0;
            while (__hip_atomic_load(tflags + wl[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
                __builtin_amdgcn_s_sleep(1);
                if (spin_expired(spins, scal)) break;
            }
        }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    __syncthreads();
}

template <bool TS>
__device__ __forceinline__ void potrf_body_sync(double* __restrict__ S, int64_t ld, int col, double* __restrict__ dinv,
                                           double* __restrict__ scal, unsigned long long* __restrict__ ts,
                                           unsigned* __restrict__ flag, double* __restrict__ smem) {
#define POTRF_TS(i) do { if (TS && threadIdx.x == 0 && blockIdx.x == 0) ts[i] = __builtin_amdgcn_s_memtime(); } while (0)
    POTRF_TS(0);
    const int64_t k0 = (int64_t)col * CB;
    // lower-triangle tiles only (80 KB, so the kernel fits beside a bulk-update workgroup on a CU):
    // element (r, c), r/16 >= c/16, at tile (r/16)(r/16+1)/2 + c/16, row r%16 (stride 17), col c%16
#define AT(r, c) smem[(((r) >> 4) * (((r) >> 4) + 1) / 2 + ((c) >> 4)) * (IB * 17) + ((r) & 15) * 17 + ((c) & 15)]
    double* Dall = smem + POTRF_NT * IB * 17;  // [8][16][17] the leaf inverses D_s (to dinv at the end)
    double* Dl = Dall;                          // the current one
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int lr = lane & 15, lk = lane >> 4;
    const int64_t dbase = (k0 / CB) * (CB / IB) * (IB * IB);
    bool ok = true;
    // store the final tiles (t, sc), t >= sc, of block column sc (diagonal tile: lower part only);
    // item i -> tile row t = sc + (i >> 7), row (i >> 3) & 15, columns 2 (i & 7)
    const __amdgpu_buffer_rsrc_t rL = block_rsrc(S + k0 * ld + k0, ((int64_t)(CB - 1) * ld + CB) * 8);
    auto store_col = [&](int sc, int t0, int nthr) {
        for (int i = t0; i < (CB / IB - sc) * 128; i += nthr) {
            const int ti = sc + (i >> 7), n = (i >> 3) & 15, m = (i & 7) * 2;
            const int64_t off = ((int64_t)(ti * IB + n) * ld + sc * IB + m) * 8;
            const double* t = smem + (ti * (ti + 1) / 2 + sc) * IB * 17 + n * 17 + m;
            if (ti > sc || m + 1 <= n) {
                double2 v;
                v.x = t[0];
                v.y = t[1];
                st_sc1(rL, off, v);
            } else if (m == n) {
                st_sc1(rL, off, t[0]);
            }
        }
    };
    {
        // wave 0 reads the rows of diagonal tile 0 straight into registers (issued first, so leaf 0
        // starts after one load latency); the other 35 lower tiles go through LDS: item i -> tile
        // p = 1 + (i >> 7), row (i >> 3) & 15, columns 2 (i & 7), all of a thread's loads in flight
        double a[IB], x[IB];
        // sc1 loads: in a merged launch the block was just updated by another workgroup
        if (wave == 0) {
#pragma unroll
            for (int h = 0; h < IB / 2; ++h) {
                const double2 v = ld_sc1(rL, ((int64_t)lr * ld + 2 * h) * 8);
                a[2 * h] = v.x;
                a[2 * h + 1] = v.y;
            }
        }
        constexpr int NQ = ((POTRF_NT - 1) * 128 + POTRF_THREADS - 1) / POTRF_THREADS;
        double2 v[NQ];
        int off[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int i = tid + POTRF_THREADS * q, p = 1 + (i >> 7), n = (i >> 3) & 15, m = (i & 7) * 2;
            int ti = 0, pp = p;
            while (pp > ti) { pp -= ti + 1; ++ti; }
            off[q] = -1;
            if (p < POTRF_NT) {
                v[q] = ld_sc1(rL, ((int64_t)(ti * IB + n) * ld + pp * IB + m) * 8);
                off[q] = p * IB * 17 + n * 17 + m;
            }
        }
        if (wave == 0) {
            POTRF_TS(1);
            ok = leaf_factor(a, x, lr);
            POTRF_TS(2);
            if (lane < IB) {
#pragma unroll
                for (int c = 0; c < IB; ++c) {
                    if (c <= lane) AT(lane, c) = a[c];
                    const double d = (c >= lane) ? x[c] : 0.0;  // (L^-1)[c][lane]
                    Dl[c * 17 + lane] = d;
                }
            }
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            if (off[q] >= 0) {
                smem[off[q]] = v[q].x;
                smem[off[q] + 1] = v[q].y;
            }
        }
    }
    for (int s = 0; s < CB / IB; ++s) {
        const int c0 = s * IB;
        __syncthreads();  // B1: L_ss, D_s in LDS; column s updated
        POTRF_TS(3 + 4 * s);
        Dl = Dall + s * IB * 17;
        if (s == CB / IB - 1) break;
        // panel solve X_t = A_ts D_s^T: wave 0 tile s+1, waves 1..7 tiles s+2..7 (with a flag, wave 4 is the
        // publisher and the other six take tiles s+2..7, one each)
        {
            const int wb = flag ? (wave < 4 ? wave : wave - 1) : wave;
            const int t0 = (wave == 0) ? s + 1 : s + 1 + wb;
            const int step = (wave == 0) ? CB : (flag ? POTRF_NW - 2 : POTRF_NW - 1);
            for (int t = t0; t < CB / IB && !(flag && wave == 4); t += step) {
                const int r0 = t * IB;
                dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int kk = 0; kk < IB; kk += 4)
                    acc = mfma(AT((r0 + lr), c0 + kk + lk), Dl[lr * 17 + kk + lk], acc);
#pragma unroll
                for (int r = 0; r < 4; ++r) AT((r0 + lk + 4 * r), c0 + lr) = acc[r];
            }
        }
        __syncthreads();  // B2: panel column s solved
        POTRF_TS(4 + 4 * s);
        if (flag && wave == 4) {
            // progressive hand-off: block column s of L and the leaf inverse D_s are final; store them
            // write-through, drain, then flag = s + 1 (the panel solves' step s needs columns < s and D_s)
            store_col(s, lane, 64);
            const __amdgpu_buffer_rsrc_t rD = block_rsrc(dinv + dbase, (CB / IB) * IB * IB * 8);
            for (int i = 2 * lane; i < IB * IB; i += 128) {
                double2 v;
                v.x = Dall[s * IB * 17 + (i >> 4) * 17 + (i & 15)];
                v.y = Dall[s * IB * 17 + (i >> 4) * 17 + (i & 15) + 1];
                st_sc1(rD, (int64_t)(s * IB * IB + i) * 8, v);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) __hip_atomic_store(flag, (unsigned)(s + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (wave == 0) {
            // next diagonal tile, then its leaf factor
            const int R = c0 + IB;
            dbl4 acc;
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[r] = AT((R + lk + 4 * r), R + lr);
#pragma unroll
            for (int kk = 0; kk < IB; kk += 4)
                acc = mfma(-AT((R + lr), c0 + kk + lk), AT((R + lr), c0 + kk + lk), acc);
#pragma unroll
            for (int r = 0; r < 4; ++r) AT((R + lk + 4 * r), R + lr) = acc[r];
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_wave_barrier();
            double a[IB], x[IB];
#pragma unroll
            for (int c = 0; c < IB; ++c) a[c] = AT((R + lr), R + c);
            POTRF_TS(5 + 4 * s);
            ok &= leaf_factor(a, x, lr);
            POTRF_TS(6 + 4 * s);
            if (lane < IB) {
#pragma unroll
                for (int c = 0; c < IB; ++c) {
                    if (c <= lane) AT((R + lane), R + c) = a[c];
                    const double v = (c >= lane) ? x[c] : 0.0;  // (L^-1)[c][lane]
                    Dall[(s + 1) * IB * 17 + c * 17 + lane] = v;
                }
            }
        } else {
            // bulk waves: the rest of the trailing update, tile rows s+2 .. 7 from the bottom (largest
            // first); the tiles of a row go in pairs sharing the A operand (two independent MFMA
            // chains), the pairs dealt round-robin over the waves
            const int nrows = CB / IB - 2 - s;
            int unit = 0;
            for (int i = 0; i < nrows; ++i) {
                const int R = (CB / IB - 1 - i) * IB;
                for (int C = c0 + IB; C <= R; C += 2 * IB, ++unit) {
                    // waves 1-3, 5-7: wave 4 shares wave 0's SIMD and stays out of the leaf's way
                    const int u6 = unit % 6;
                    if (u6 + (u6 >= 3 ? 2 : 1) != wave) continue;
                    const bool two = C + IB <= R;
                    dbl4 acc1, acc2 = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc1[r] = AT((R + lk + 4 * r), C + lr);
                    if (two)
#pragma unroll
                        for (int r = 0; r < 4; ++r) acc2[r] = AT((R + lk + 4 * r), C + IB + lr);
#pragma unroll
                    for (int kk = 0; kk < IB; kk += 4) {
                        const double av = -AT((R + lr), c0 + kk + lk);
                        acc1 = mfma(av, AT((C + lr), c0 + kk + lk), acc1);
                        if (two) acc2 = mfma(av, AT((C + IB + lr), c0 + kk + lk), acc2);
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) AT((R + lk + 4 * r), C + lr) = acc1[r];
                    if (two)
#pragma unroll
                        for (int r = 0; r < 4; ++r) AT((R + lk + 4 * r), C + IB + lr) = acc2[r];
                }
            }
            if (!flag) store_col(s, tid - 64, POTRF_THREADS - 64);  // block column s is final: written behind the update
        }
    }
    if (!ok && lane == 0) pivot_failed(scal, k0);
    store_col(CB / IB - 1, tid, POTRF_THREADS);
    {   // the leaf inverses, row-major 16x16 each, two per thread-store (with a flag only D_7 is left)
        const __amdgpu_buffer_rsrc_t rD = block_rsrc(dinv + dbase, (CB / IB) * IB * IB * 8);
        for (int i = 2 * tid + (flag ? (CB / IB - 1) * IB * IB : 0); i < (CB / IB) * IB * IB; i += 2 * POTRF_THREADS) {
            double2 v;
            v.x = Dall[(i >> 8) * IB * 17 + ((i >> 4) & 15) * 17 + (i & 15)];
            v.y = Dall[(i >> 8) * IB * 17 + ((i >> 4) & 15) * 17 + (i & 15) + 1];
            st_sc1(rD, (int64_t)i * 8, v);
        }
    }
    POTRF_TS(40);
    if (flag) {  // publish: every storing wave drains, the barrier, then one lane's flag
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_store(flag, (unsigned)(CB / IB), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#undef AT
#undef POTRF_TS
}

__device__ __forceinline__ void spin_ge(const unsigned* p, unsigned v, double* __restrict__ scal) {
    unsigned spins = 0;
    while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < v) {
        __builtin_amdgcn_s_sleep(1);
        if (spin_expired(spins, scal)) break;  // hand-off timeout (host reports it)
    }
}

// tile sets of a fused diagonal update (tiles (a, b), a >= b, in row order): 0 all 36 lower tiles, 1 those
// of tile columns < FLOW_CSPLIT (the diagonal workgroup's share when split), 2 the others (the helper's)
__host__ __device__ constexpr bool fset_has(int set, int b) { return set == 0 || (set == 1) == (b < FLOW_CSPLIT); }
__host__ __device__ constexpr int fset_count(int set) {
    int n = 0;
    for (int a = 0; a < CB / IB; ++a)
        for (int b = 0; b <= a; ++b) n += fset_has(set, b) ? 1 : 0;
    return n;
}
__device__ __forceinline__ void fset_tile(int set, int idx, int& ta, int& tb) {  // (0, 0) past the end
    ta = tb = 0;
    int n = 0;
    for (int a = 0; a < CB / IB; ++a)
        for (int b = 0; b <= a; ++b)
            if (fset_has(set, b)) {
                if (n == idx) { ta = a; tb = b; }
                ++n;
            }
}


// potrf_body (dataflow): factor the 128x128 diagonal block of column col (512 threads); flag != nullptr:
// publish it column by column (k_panel hand-off).  No workgroup barriers after the load: the waves
// coordinate through LDS counters (workgroup-scope release / acquire), so wave 0 runs the critical
// chain back to back:
//   wave 0      leaf s (16x16 factor + inverse in registers, lane i = row i, DPP broadcasts; its
//               columns stored to LDS as they finalise) -> panel tile (s+1, s) = A D_s' -> diagonal
//               tile (s+1, s+1) -= X X' (v_mfma_f64_16x16x4_f64) -> leaf s+1
//   bulk waves  (1-3, 5-7) after leaf s: the panel tiles (r, s), r >= s+2, then the trailing update of
//               rows >= s+2 by column s, row s+2 (wave 0's next operands) first
//   wave 4      (wave 0's SIMD, mostly asleep) stores block column s and D_s once column s is solved,
//               and with a flag publishes them
// Every wait points to work that does not wait for the waiter, so the chain always progresses; the
// polls are bounded (scal[1] = -1 on timeout, reported by the host).
// PRE: the block's lower tiles are already in LDS (k_chol_flow's diagonal workgroup updated them there)
// hpart (flag hflag): the split helper's partial of the tiles of tile columns >= FLOW_CSPLIT (fset 2 order,
// 16 x 16 row-major each), added by the bulk waves at their step FLOW_CSPLIT - 2, between the trailing
// updates of the step before (every one done) and their own; nothing reads those tiles earlier (wave 0's
// step s touches tiles (s+1, s), (s+1, s+1); wave 4 stores block column s after step s)
template <bool TS, bool PRE = false>
__device__ __forceinline__ void potrf_body(double* __restrict__ S, int64_t ld, int col, double* __restrict__ dinv,
                                           double* __restrict__ scal, unsigned long long* __restrict__ ts,
                                           unsigned* __restrict__ flag, double* __restrict__ smem,
                                           uint64_t* __restrict__ pubts = nullptr, const double* __restrict__ hpart = nullptr,
                                           const unsigned* __restrict__ hflag = nullptr) {
#define POTRF_TS(i) do { if (TS && threadIdx.x == 0 && blockIdx.x == 0) ts[i] = __builtin_amdgcn_s_memtime(); } while (0)
#define BULK_TS(i) do { if (TS && threadIdx.x == 64 && blockIdx.x == 0) ts[i] = __builtin_amdgcn_s_memtime(); } while (0)
    POTRF_TS(0);
    const int64_t k0 = (int64_t)col * CB;
#define AT(r, c) smem[(((r) >> 4) * (((r) >> 4) + 1) / 2 + ((c) >> 4)) * (IB * 17) + ((r) & 15) * 17 + ((c) & 15)]
    double* Dall = smem + POTRF_NT * IB * 17;  // [8][16][17] the leaf inverses D_s
    int* sy = reinterpret_cast<int*>(Dall + (CB / IB) * IB * 17);
    int* s_leaf = sy;       // leaves factored (L_ss and D_s in LDS; leaf 0 before the barrier)
    int* s_pc = sy + 1;     // [7] panel tiles of column s solved (complete: 7 - s)
    int* s_bc = sy + 8;     // [6] bulk waves done with the trailing update of step s (complete: 6)
    int* s_cc = sy + 16;    // [6] row s+2 (tiles (s+2, s+1), (s+2, s+2)) updated by column s
    int* s_add = sy + 14;   // bulk waves done adding the split helper's partial
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int lr = lane & 15, lk = lane >> 4;
    const int64_t dbase = (k0 / CB) * (CB / IB) * (IB * IB);
    constexpr int NBULK = 6;
    bool ok = true;
    auto wait_ge = [&](int* p, int v) {  // bounded (a lost update would be a bug: reported, not hung)
        unsigned spins = 0;
        while (__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < v) {
            __builtin_amdgcn_s_sleep(1);
            if (spin_expired(spins, scal)) break;
        }
    };
    auto bump = [&](int* p) {  // after this wave's LDS writes
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) __hip_atomic_fetch_add(p, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    if (tid < 32) sy[tid] = 0;
    const __amdgpu_buffer_rsrc_t rL = block_rsrc(S + k0 * ld + k0, ((int64_t)(CB - 1) * ld + CB) * 8);
    // wave 0's leaf s: column j of L and row j of D_s to LDS as soon as they are final
    double a[IB], x[IB];
    // (branch-free, so the scheduler can overlap them with the pivot chain: all four 16-lane rows of
    // the wave hold the same leaf and store the same values; a[j] of lanes < j lands in the unused
    // upper triangle of the diagonal tile, and x[j] is exactly zero there: (L^-1)[j][lane] = 0, j < lane)
    auto leaf = [&](int s) {
        const int R = s * IB;
        double* Lw = &AT((R + lr), R);
        double* Dw = Dall + s * IB * 17 + lr;
        return leaf_factor(a, x, lr, [&](int j) {
            Lw[j] = a[j];
            Dw[j * 17] = x[j];  // (L^-1)[j][lane]
        });
    };
    if constexpr (PRE) {
        if (wave == 0) {
#pragma unroll
            for (int c = 0; c < IB; ++c) a[c] = AT(lr, c);
            ok = leaf(0);
            // FBA_PANEL_TRACE (k_chol_flow's record stamps, pubts = record + 16): leaf 0 factored
            if (pubts && lane == 0) pubts[-13] = wall_clock64();
        }
    } else {
        // wave 0 reads the rows of diagonal tile 0 straight into registers and factors leaf 0 while the
        // other 35 lower tiles are on their way into LDS (sc1 loads: in a merged launch the block was
        // just updated by another workgroup); item i -> tile p = 1 + (i >> 7), row (i >> 3) & 15,
        // columns 2 (i & 7)
        if (wave == 0) {
#pragma unroll
            for (int h = 0; h < IB / 2; ++h) {
                const double2 v = ld_sc1(rL, ((int64_t)lr * ld + 2 * h) * 8);
                a[2 * h] = v.x;
                a[2 * h + 1] = v.y;
            }
        }
        constexpr int NQ = ((POTRF_NT - 1) * 128 + POTRF_THREADS - 1) / POTRF_THREADS;
        double2 v[NQ];
        int off[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int i = tid + POTRF_THREADS * q, p = 1 + (i >> 7), n = (i >> 3) & 15, m = (i & 7) * 2;
            int ti = 0, pp = p;
            while (pp > ti) { pp -= ti + 1; ++ti; }
            off[q] = -1;
            if (p < POTRF_NT) {
                v[q] = ld_sc1(rL, ((int64_t)(ti * IB + n) * ld + pp * IB + m) * 8);
                off[q] = p * IB * 17 + n * 17 + m;
            }
        }
        if (wave == 0) {
            POTRF_TS(1);
            ok = leaf(0);
            POTRF_TS(2);
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            if (off[q] >= 0) {
                smem[off[q]] = v[q].x;
                smem[off[q] + 1] = v[q].y;
            }
        }
    }
    __syncthreads();  // all tiles, leaf 0 and the zeroed counters in LDS
    if (tid == 0) __hip_atomic_store(s_leaf, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (PRE && pubts && tid == 0) pubts[-10] = wall_clock64();  // FBA_PANEL_TRACE: past the barrier
    POTRF_TS(3);
    if (wave == 0) {
        // the critical chain
        for (int s = 0; s < CB / IB - 1; ++s) {
            const int c0 = s * IB, R = c0 + IB;
            if (s > 0) wait_ge(s_cc + s - 1, 1);  // row s+1 updated through column s-1
            POTRF_TS(4 + 4 * s);
            const double* Dl = Dall + s * IB * 17;
            const dbl4 z = dbl4{0.0, 0.0, 0.0, 0.0};
            dbl4 x1 = z, x2 = z, d, d2 = z;
#pragma unroll
            for (int r = 0; r < 4; ++r) d[r] = AT((R + lk + 4 * r), R + lr);
            // X' = D_s A' (the operands of X = A D_s' swapped): lane (lr, lk) gets xt[r] = X[lr][4r + lk],
            // the diagonal update's operand as it stands (no LDS round trip before it); two accumulators
            // halve each dependent MFMA chain
#pragma unroll
            for (int kk = 0; kk < IB; kk += 8) {
                x1 = mfma(Dl[lr * 17 + kk + lk], AT((R + lr), c0 + kk + lk), x1);
                x2 = mfma(Dl[lr * 17 + kk + 4 + lk], AT((R + lr), c0 + kk + 4 + lk), x2);
            }
            dbl4 xt;
#pragma unroll
            for (int r = 0; r < 4; ++r) xt[r] = x1[r] + x2[r];
#pragma unroll
            for (int kk = 0; kk < 4; kk += 2) {  // C -= X X'
                d = mfma(-xt[kk], xt[kk], d);
                d2 = mfma(-xt[kk + 1], xt[kk + 1], d2);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) AT((R + lr), c0 + 4 * r + lk) = xt[r];  // X: panel tile (s+1, s)
            bump(s_pc + s);
#pragma unroll
            for (int r = 0; r < 4; ++r) AT((R + lk + 4 * r), R + lr) = d[r] + d2[r];
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int c = 0; c < IB; ++c) a[c] = AT((R + lr), R + c);
            POTRF_TS(5 + 4 * s);
            ok &= leaf(s + 1);
            POTRF_TS(6 + 4 * s);
            bump(s_leaf);
            POTRF_TS(7 + 4 * s);
        }
    } else if (wave != 4) {
        // bulk waves: the whole schedule unrolled (every tile index a compile-time constant, one
        // uniform branch per unit on its owner), each unit's LDS operands loaded before its MFMAs
        const int b = wave < 4 ? wave - 1 : wave - 2;
        // C(R, C) -= X(R) X(C)' [and C(R, C + 16) -= X(R) X(C + 16)'], K = 16 from column c0
        auto unit = [&](const int c0, const int R, const int C, const bool two) {
            dbl4 acc1, acc2;
            double av[4], b1[4], b2[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) acc1[r] = AT((R + lk + 4 * r), C + lr);
            if (two)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc2[r] = AT((R + lk + 4 * r), C + IB + lr);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                av[k] = -AT((R + lr), c0 + 4 * k + lk);
                b1[k] = AT((C + lr), c0 + 4 * k + lk);
                if (two) b2[k] = AT((C + IB + lr), c0 + 4 * k + lk);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                acc1 = mfma(av[k], b1[k], acc1);
                if (two) acc2 = mfma(av[k], b2[k], acc2);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) AT((R + lk + 4 * r), C + lr) = acc1[r];
            if (two)
#pragma unroll
                for (int r = 0; r < 4; ++r) AT((R + lk + 4 * r), C + IB + lr) = acc2[r];
        };
#pragma unroll
        for (int s = 0; s < CB / IB - 2; ++s) {
            const int c0 = s * IB;
            wait_ge(s_leaf, s + 1);                   // L_ss, D_s
            BULK_TS(41 + 3 * s);
            if (s > 0) wait_ge(s_bc + s - 1, NBULK);  // every update of step s-1
            BULK_TS(42 + 3 * s);
            // the split helper's partial: this wave's tiles h = b + 6 m (15 in all) in flight during the
            // panel tile, then added; every bulk wave polls the flag itself before its loads
            constexpr int NH = fset_count(2), HM = (NH + NBULK - 1) / NBULK;
            static_assert(FLOW_CSPLIT >= 2 && FLOW_CSPLIT < CB / IB, "split step");
            double2 hv[HM][2];
            if (hpart && s == FLOW_CSPLIT - 2) {
                spin_ge(hflag, 1u, scal);
                const __amdgpu_buffer_rsrc_t rH = block_rsrc(hpart, NH * IB * IB * 8);
#pragma unroll
                for (int m = 0; m < HM; ++m)
                    if (b + NBULK * m < NH)
#pragma unroll
                        for (int e = 0; e < 2; ++e)
                            hv[m][e] = ld_sc1(rH, (int64_t)((b + NBULK * m) * IB * IB + 2 * (lane + 64 * e)) * 8);
            }
            if (b < CB / IB - 2 - s) {                // panel tile (s+2+b, s)
                const int r0 = (s + 2 + b) * IB;
                const double* Dl = Dall + s * IB * 17;
                double av[4], bv[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    av[k] = AT((r0 + lr), c0 + 4 * k + lk);
                    bv[k] = Dl[lr * 17 + 4 * k + lk];
                }
                dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int k = 0; k < 4; ++k) acc = mfma(av[k], bv[k], acc);
#pragma unroll
                for (int r = 0; r < 4; ++r) AT((r0 + lk + 4 * r), c0 + lr) = acc[r];
                bump(s_pc + s);
                if (PRE && pubts && s == 0 && b == 0 && lane == 0) pubts[-9] = wall_clock64();  // panel tile (2, 0)
            }
            if (hpart && s == FLOW_CSPLIT - 2) {
#pragma unroll
                for (int m = 0; m < HM; ++m)
                    if (b + NBULK * m < NH) {
                        int ha, hb;
                        fset_tile(2, b + NBULK * m, ha, hb);
#pragma unroll
                        for (int e = 0; e < 2; ++e) {
                            const int x = 2 * (lane + 64 * e), hr = IB * ha + (x >> 4), hc = IB * hb + (x & 15);
                            AT(hr, hc) += hv[m][e].x;
                            AT(hr, hc + 1) += hv[m][e].y;
                        }
                    }
                bump(s_add);
                wait_ge(s_add, NBULK);  // every tile final before this step's trailing updates
            }
            wait_ge(s_pc + s, CB / IB - 1 - s);  // column s solved
            // trailing update of rows s+2 .. 7 by column s: row s+2 (wave 0's next panel tile and
            // diagonal tile) on bulk wave 0 first, then the other rows from the bottom, tiles in pairs
            // sharing the A operand, dealt round-robin from bulk wave 1 on
            if (b == 0) {
                unit(c0, (s + 2) * IB, (s + 1) * IB, true);
                bump(s_cc + s);
                BULK_TS(43 + 3 * s);
            }
            int u = 0;
#pragma unroll
            for (int i = CB / IB - 1; i >= s + 3; --i)
#pragma unroll
                for (int C = c0 + IB; C <= i * IB; C += 2 * IB, ++u)
                    if ((1 + u) % NBULK == b) unit(c0, i * IB, C, C + IB <= i * IB);
            bump(s_bc + s);
        }
    } else {
        // wave 4: block column s (tiles (s..7, s)) and D_s are final once column s is solved; per column
        // every LDS read is issued before the stores (compile-time trip counts: the reads of a column
        // are one batch, not a read-wait-store round per item, on the SIMD wave 0's chain runs on)
        const __amdgpu_buffer_rsrc_t rD = block_rsrc(dinv + dbase, (CB / IB) * IB * IB * 8);
        bulk_for(std::make_integer_sequence<int, CB / IB>{}, [&](auto sc) {
            constexpr int s = decltype(sc)::value;
            constexpr int NI = (CB / IB - s) * 2;  // 16-B items per lane: 128 per tile, 64 lanes
            if constexpr (s < CB / IB - 1) wait_ge(s_pc + s, CB / IB - 1 - s);
            else wait_ge(s_leaf, CB / IB);
            double2 v[NI + 2];
#pragma unroll
            for (int u = 0; u < NI; ++u) {
                const int i = lane + 64 * u, ti = s + (i >> 7), n = (i >> 3) & 15, m = (i & 7) * 2;
                const double* t = smem + (ti * (ti + 1) / 2 + s) * IB * 17 + n * 17 + m;
                v[u].x = t[0];
                v[u].y = t[1];
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int i = 2 * lane + 128 * u;
                v[NI + u].x = Dall[s * IB * 17 + (i >> 4) * 17 + (i & 15)];
                v[NI + u].y = Dall[s * IB * 17 + (i >> 4) * 17 + (i & 15) + 1];
            }
#pragma unroll
            for (int u = 0; u < NI; ++u) {
                const int i = lane + 64 * u, ti = s + (i >> 7), n = (i >> 3) & 15, m = (i & 7) * 2;
                const int64_t off = ((int64_t)(ti * IB + n) * ld + s * IB + m) * 8;
                if (ti > s || m + 1 <= n) st_sc1(rL, off, v[u]);
                else if (m == n) st_sc1(rL, off, v[u].x);
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) st_sc1(rD, (int64_t)(s * IB * IB + 2 * lane + 128 * u) * 8, v[NI + u]);
            if (flag) {
                if (pubts && lane == 0) pubts[8 + s] = wall_clock64();  // FBA_PANEL_TRACE: column s solved
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0) __hip_atomic_store(flag, (unsigned)(s + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (pubts && lane == 0) pubts[16 + s] = wall_clock64();  // ... and published
            }
        });
    }
    if (!ok && lane == 0) pivot_failed(scal, k0);
    POTRF_TS(40);
#undef AT
#undef POTRF_TS
#undef BULK_TS
}

template <bool TS>
__global__ __launch_bounds__(POTRF_THREADS) void k_potrf128(double* __restrict__ S, int64_t ld, const int32_t* __restrict__ cols,
                                                            double* __restrict__ dinv, double* __restrict__ scal,
                                                            unsigned long long* __restrict__ ts) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    potrf_body<TS>(S, ld, cols[blockIdx.x], dinv, scal, ts, nullptr, smem);
}


// ------------------------------------------------------------------------------------------------
// k_trsm128: one workgroup per 64-row half of a panel block (column k, block row r), r in the panel rows of
// column k:
//   X = A L^-T by blocked substitution, X_s = (A_s - sum_{t<s} X_t L_st^T) D_s^T.
// 256 threads = 4 waves x 16 rows.  L_kk was just written by another CU, so its reads are far-cache
// latency bound: the whole workgroup stages the 28 off-diagonal 16x16 tiles of L_kk and the eight
// D_s into LDS with one round of loads (issued together with the panel rows), after which each wave
// runs its eight sub-steps out of LDS only.
// ------------------------------------------------------------------------------------------------
constexpr int TRSM_NT = (CB / IB) * (CB / IB - 1) / 2;  // 28 off-diagonal tiles
constexpr size_t TRSM_LDS = sizeof(double) * (4 * IB * LDA + 4 * IB * 17 + (TRSM_NT + CB / IB) * IB * 17 + 4);  // + the loaders' column flags

// one substitution step of a wave's 16 panel rows: X_s = (A_s - sum_{t<s} X_t L_st^T) D_s^T
__device__ __forceinline__ void trsm_step(const int s, double* __restrict__ Xw, double* __restrict__ Tw,
                                          const double* __restrict__ Lt, const double* __restrict__ Dt, int lr, int lk) {
    const int c0 = s * IB;
    // Z = A_s - sum_{t<s} X_t L_st^T : output 16x16, K = 16 s.  All operands of the step are read
    // from LDS in one batch, then two independent MFMA chains.
    double av[CB / 4], bv[CB / 4];
#pragma unroll
    for (int t = 0; t < s; ++t) {
        const double* Lst = Lt + (s * (s - 1) / 2 + t) * IB * 17;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {  // B[k][n] = L[c0+n][t*16+k]
            av[4 * t + kk] = Xw[lr * LDA + t * IB + 4 * kk + lk];
            bv[4 * t + kk] = Lst[lr * 17 + 4 * kk + lk];
        }
    }
    dbl4 p0 = dbl4{0.0, 0.0, 0.0, 0.0}, p1 = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < 4 * s; q += 2) {
        p0 = mfma(av[q], bv[q], p0);
        p1 = mfma(av[q + 1], bv[q + 1], p1);
    }
    dbl4 acc;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = Xw[(lk + 4 * r) * LDA + c0 + lr] - (p0[r] + p1[r]);
    // Z (D layout) -> LDS, then X_s = Z D_s^T
#pragma unroll
    for (int r = 0; r < 4; ++r) Tw[(lk + 4 * r) * 17 + lr] = acc[r];
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    dbl4 out = dbl4{0.0, 0.0, 0.0, 0.0};
    const double* Ds = Dt + s * IB * 17;
#pragma unroll
    for (int kk = 0; kk < IB; kk += 4) out = mfma(Tw[lr * 17 + kk + lk], Ds[lr * 17 + kk + lk], out);
#pragma unroll
    for (int r = 0; r < 4; ++r) Xw[(lk + 4 * r) * LDA + c0 + lr] = out[r];
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void trsm_store(double* __restrict__ S, int64_t ld, int64_t rbase, int64_t k0,
                                           const double* __restrict__ Xw, int lane) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int idx = lane + 64 * q, r = idx >> 6, c = (idx & 63) * 2;
        double2 v;
        v.x = Xw[r * LDA + c];
        v.y = Xw[r * LDA + c + 1];
        *reinterpret_cast<double2*>(S + (rbase + r) * ld + k0 + c) = v;
    }
}

// trsm_body: threads 0..255 (4 waves x 16 rows) solve one record; flag != nullptr: the factor of
// column k comes from a potrf workgroup of the same launch (wait for its flag, sc1 loads); the threads
// 256.. of a 512-thread workgroup only take part in the barriers
__device__ __forceinline__ void trsm_body(double* __restrict__ S, int64_t ld, const int32_t* __restrict__ rec,
                                          const double* __restrict__ dinv, const unsigned* __restrict__ flag,
                                          double* __restrict__ scal, double* __restrict__ smem, bool progressive,
                                          uint64_t* __restrict__ tr = nullptr) {
    double* X = smem;                       // [4][IB][LDA]   panel rows of each wave
    double* T = X + 4 * IB * LDA;           // [4][IB][17]    per-wave 16x16 staging
    double* Lt = T + 4 * IB * 17;           // [28][IB][17]   L_st, p = s(s-1)/2 + t
    double* Dt = Lt + TRSM_NT * IB * 17;    // [8][IB][17]    D_s
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int lr = lane & 15, lk = lane >> 4;
    const bool worker = tid < 256;
    // record (column k, 2 r + h): rows 64 h .. 64 h + 63 of panel block (r, k)
    const int64_t k0 = (int64_t)rec[0] * CB;
    const int rh = rec[1];
    const int64_t rbase = (int64_t)(rh >> 1) * CB + (rh & 1) * 64 + wave * IB;
    double* Xw = X + wave * IB * LDA;
    double* Tw = T + wave * IB * 17;
    const double* L = S + k0 * ld + k0;
    const double* Dk = dinv + (k0 / CB) * (CB / IB) * (IB * IB);
    if (worker) {  // the panel rows, issued first (sc1: in a merged launch just updated by another workgroup)
        const __amdgpu_buffer_rsrc_t rA = block_rsrc(S + rbase * ld + k0, ((int64_t)(IB - 1) * ld + CB) * 8);
        double2 v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int idx = lane + 64 * q, r = idx >> 6, c = (idx & 63) * 2;
            v[q] = ld_sc1(rA, ((int64_t)r * ld + c) * 8);
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int idx = lane + 64 * q, r = idx >> 6, c = (idx & 63) * 2;
            Xw[r * LDA + c] = v[q].x;
            Xw[r * LDA + c + 1] = v[q].y;
        }
    }
    const __amdgpu_buffer_rsrc_t rL = block_rsrc(L, ((int64_t)(CB - 1) * ld + CB) * 8);
    const __amdgpu_buffer_rsrc_t rD = block_rsrc(Dk, (CB / IB) * IB * IB * 8);
    auto wait_flag = [&](unsigned v) {  // one lane polls, relaxed, bounded; then the whole workgroup
        if (tid == 0) {
            unsigned spins = 0;
            while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < v) {
                __builtin_amdgcn_s_sleep(1);
                if (spin_expired(spins, scal)) break;  // hand-off timeout (host reports it)
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep the payload loads below the poll
        __syncthreads();
    };
    if (flag && progressive) {
        // progressive hand-off (k_panel): step st needs block columns < st of L_kk and D_st, final
        // once flag >= st + 1.  Waves 4-7 (idle otherwise: the solve uses waves 0-3) are loaders, wave
        // 4 + t % 4 for block column t: it polls the flag, copies the column (tiles (r, t), r > t, and
        // D_t; sc1 loads, 16 per lane in flight) into LDS and raises the column's LDS flag.  Four
        // columns are in flight at once, so the load latency overlaps both the factorisation and the
        // substitution steps; the solving waves wait on the LDS flags only.
        int* s_col = reinterpret_cast<int*>(Dt + (CB / IB) * IB * 17);  // [8] column t in LDS
        if (tid < CB / IB) s_col[tid] = 0;
        __syncthreads();  // the panel rows are in LDS, the flags are zero
        if (!worker) {
            for (int t = wave - 4; t < CB / IB; t += 4) {
                unsigned spins = 0;
                while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)(t + 1)) {
                    __builtin_amdgcn_s_sleep(1);
                    if (spin_expired(spins, scal)) break;  // (hand-off timeout or abort: reported by the host)
                }
                double2 v[16];
                double* dst[16];
#pragma unroll
                for (int q = 0; q < 16; ++q) {  // items (8 - t) * 128 double2
                    const int i = lane + 64 * q, u = i >> 7, n = (i >> 3) & 15, kc = (i & 7) * 2;
                    dst[q] = nullptr;
                    if (u < CB / IB - 1 - t) {  // tile (r, t), r = t + 1 + u
                        const int r = t + 1 + u;
                        v[q] = ld_sc1(rL, ((int64_t)(r * IB + n) * ld + t * IB + kc) * 8);
                        dst[q] = Lt + ((r * (r - 1) / 2 + t) * IB + n) * 17 + kc;
                    } else if (u == CB / IB - 1 - t) {  // D_t
                        v[q] = ld_sc1(rD, (int64_t)(t * IB * IB + n * IB + kc) * 8);
                        dst[q] = Dt + (t * IB + n) * 17 + kc;
                    }
                }
#pragma unroll
                for (int q = 0; q < 16; ++q)
                    if (dst[q]) {
                        dst[q][0] = v[q].x;
                        dst[q][1] = v[q].y;
                    }
                __builtin_amdgcn_s_waitcnt(0xC07F);  // this wave's LDS writes done
                __builtin_amdgcn_wave_barrier();
                if (lane == 0) __hip_atomic_store(s_col + t, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (tr && lane == 0 && t == CB / IB - 1) tr[1] = wall_clock64();  // FBA_PANEL_TRACE: last column in
            }
        } else {
#pragma unroll
            for (int st = 0; st < CB / IB; ++st) {
                unsigned sp = 0;
                while (__hip_atomic_load(s_col + st, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) {
                    __builtin_amdgcn_s_sleep(1);
                    if (spin_expired(sp, scal)) break;
                }
                trsm_step(st, Xw, Tw, Lt, Dt, lr, lk);
                if (tr && tid == 0 && st == CB / IB - 2) tr[5] = wall_clock64();
            }
            if (tr && tid == 0) tr[6] = wall_clock64();
            trsm_store(S, ld, rbase, k0, Xw, lane);
        }
        return;
    }
    if (flag) wait_flag((unsigned)(CB / IB));  // the whole factor
    if (worker) {  // the factor: off-diagonal tiles of L_kk and the leaf inverses, sc1 loads
        double2 lv[14], dv[4];
        // off-diagonal tiles: item i -> tile p = i >> 7, row n = (i >> 3) & 15, columns 2*(i & 7)
#pragma unroll
        for (int q = 0; q < 14; ++q) {
            const int i = tid + 256 * q, p = i >> 7, n = (i >> 3) & 15, kc = (i & 7) * 2;
            int sr = 1, pp = p;
            while (pp >= sr) { pp -= sr; ++sr; }
            lv[q] = ld_sc1(rL, ((int64_t)(sr * IB + n) * ld + pp * IB + kc) * 8);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) dv[q] = ld_sc1(rD, (int64_t)(2 * (tid + 256 * q)) * 8);
#pragma unroll
        for (int q = 0; q < 14; ++q) {
            const int i = tid + 256 * q, p = i >> 7, n = (i >> 3) & 15, kc = (i & 7) * 2;
            Lt[(p * IB + n) * 17 + kc] = lv[q].x;
            Lt[(p * IB + n) * 17 + kc + 1] = lv[q].y;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int e = 2 * (tid + 256 * q), sd = e >> 8, n = (e >> 4) & 15, kc = e & 15;
            Dt[(sd * IB + n) * 17 + kc] = dv[q].x;
            Dt[(sd * IB + n) * 17 + kc + 1] = dv[q].y;
        }
    }
    __syncthreads();
    if (!worker) return;
#pragma unroll
    for (int st = 0; st < CB / IB; ++st) trsm_step(st, Xw, Tw, Lt, Dt, lr, lk);
    trsm_store(S, ld, rbase, k0, Xw, lane);
}

__global__ __launch_bounds__(256) void k_trsm128(double* __restrict__ S, int64_t ld, const int32_t* __restrict__ tasks,
                                                 const double* __restrict__ dinv) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    trsm_body(S, ld, tasks + 2 * blockIdx.x, dinv, nullptr, nullptr, smem, false);
}

// ------------------------------------------------------------------------------------------------
// k_syrk_multi: the trailing updates of one level, one 64x64 output quarter per workgroup (task record,
// Sched): C(i,j) -= sum_k X_ik X_jk^T over the task's source columns k (ascending), or, for a split
// target, the partial sum of a group of sources into a scratch quarter (the last group to arrive adds
// the groups in slot order): the result does not depend on the schedule.  K = 128 per source column staged through
// LDS in 32-deep slices, the next slice prefetched into registers while the MFMAs of the current one
// run.
// ------------------------------------------------------------------------------------------------
constexpr int KS = 32;
constexpr int LDK = 34;   // LDS stride of a 32-deep slice: bank = (4r + 2k) mod 64, conflict-free

// syrk_body: one quarter task; threads 0..255 work, threads 256.. (a 512-thread k_panel workgroup) only
// take part in the barriers.  tflags != nullptr: the task runs inside the next level's k_panel, so the
// target quarter is written through (sc1) and its completion flag raised for the potrf / panel-solve
// workgroups of that launch that consume it.
__device__ __forceinline__ void syrk_body(double* __restrict__ S, int64_t ld, const int32_t* __restrict__ tk,
                                          const int32_t* __restrict__ src, double* __restrict__ P,
                                          const int32_t* __restrict__ comb, unsigned* __restrict__ cnt,
                                          unsigned* __restrict__ tflags, double* __restrict__ smem) {
    double (*As)[LDK] = reinterpret_cast<double (*)[LDK]>(smem);
    double (*Bs)[LDK] = reinterpret_cast<double (*)[LDK]>(smem + 64 * LDK);
    unsigned* last = reinterpret_cast<unsigned*>(smem + 128 * LDK);
    const int64_t bi = tk[0], bj = tk[1];
    const int qr = tk[2] >> 1, qc = tk[2] & 1, s0 = tk[3], slot = tk[5];
    const int nsl = 4 * (tk[4] - s0);
    const int32_t* ks_src = src + s0;
    const int64_t r0 = bi * CB + qr * 64, c0 = bj * CB + qc * 64;
    const int tid = threadIdx.x, wave = (tid & 255) >> 6, lane = tid & 63;
    const bool worker = tid < 256;
    const int lr = lane & 15, lk = lane >> 4;
    const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
    // output: the C quarter in place, or scratch quarter `slot` (row-major 64x64, starts from zero)
    double* Cp = slot < 0 ? S + (r0 + wr + lk) * ld + c0 + wc + lr : P + (int64_t)slot * 4096 + (wr + lk) * 64 + wc + lr;
    const int64_t ldc = slot < 0 ? ld : 64;
    dbl4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[a][b][r] = (slot < 0 && worker) ? Cp[(a * 16 + 4 * r) * ldc + b * 16] : 0.0;
    // loader mapping: thread t of the first 256 -> rows (t >> 4) + 16 h, columns 2 (t & 15), 2 (t & 15) + 1 of
    // the 32-deep slice: one wave instruction reads four whole 256-B row slices (8 cache lines)
    const int rr = (tid & 255) >> 4, cc = (tid & 15) * 2;
    const double* ga = S + (r0 + rr) * ld + cc;
    const double* gb = S + (c0 + rr) * ld + cc;
    double2 pa[4], pb[4];
    if (worker) {
        const int64_t kc = (int64_t)ks_src[0] * CB;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            pa[h] = *reinterpret_cast<const double2*>(ga + (int64_t)(16 * h) * ld + kc);
            pb[h] = *reinterpret_cast<const double2*>(gb + (int64_t)(16 * h) * ld + kc);
        }
    }
    for (int sl = 0; sl < nsl; ++sl) {
        __syncthreads();
        if (worker) {
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                As[rr + 16 * h][cc] = pa[h].x; As[rr + 16 * h][cc + 1] = pa[h].y;
                Bs[rr + 16 * h][cc] = pb[h].x; Bs[rr + 16 * h][cc + 1] = pb[h].y;
            }
        }
        __syncthreads();
        if (worker) {
            if (sl + 1 < nsl) {
                const int64_t kc = (int64_t)ks_src[(sl + 1) >> 2] * CB + ((sl + 1) & 3) * KS;
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    pa[h] = *reinterpret_cast<const double2*>(ga + (int64_t)(16 * h) * ld + kc);
                    pb[h] = *reinterpret_cast<const double2*>(gb + (int64_t)(16 * h) * ld + kc);
                }
            }
#pragma unroll
            for (int kk = 0; kk < KS; kk += 4) {
                double av[2], bv[2];
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    av[q] = -As[wr + q * 16 + lr][kk + lk];
                    bv[q] = Bs[wc + q * 16 + lr][kk + lk];
                }
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int b = 0; b < 2; ++b) acc[a][b] = mfma(av[a], bv[b], acc[a][b]);
            }
        }
    }
    const __amdgpu_buffer_rsrc_t rC = block_rsrc(S + r0 * ld + c0, ((int64_t)63 * ld + 64) * 8);
    if (slot < 0) {
        if (worker) {
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        if (tflags)
                            st_sc1(rC, ((int64_t)(wr + lk + a * 16 + 4 * r) * ld + wc + lr + b * 16) * 8, acc[a][b][r]);
                        else
                            Cp[(a * 16 + 4 * r) * ldc + b * 16] = acc[a][b][r];
                    }
        }
        if (tflags) {  // publish the quarter
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) __hip_atomic_store(tflags + tk[7], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    // split target: this group's partial goes to its scratch quarter write-through; the group that
    // arrives last (agent-scope counter) adds all groups' partials to C in slot order -- the same
    // arithmetic as a separate combine launch, so the result does not depend on the arrival order
    if (worker) {
        const __amdgpu_buffer_rsrc_t rP = block_rsrc(P + (int64_t)slot * 4096, 4096 * 8);
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    st_sc1(rP, (int64_t)((wr + lk + a * 16 + 4 * r) * 64 + wc + lr + b * 16) * 8, acc[a][b][r]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int32_t* cb = comb + Sched::COMB_REC * tk[6];
    if (tid == 0)
        *last = __hip_atomic_fetch_add(cnt + tk[6], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(cb[4] - 1);
    __syncthreads();
    if (!*last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const int first = cb[3], n = cb[4];
    if (worker) {
        double2 v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = 2 * (tid + 256 * q), r = e >> 6, cl = e & 63;
            v[q] = *reinterpret_cast<const double2*>(S + (r0 + r) * ld + c0 + cl);
        }
        for (int g = 0; g < n; ++g) {
            const __amdgpu_buffer_rsrc_t rg = block_rsrc(P + (int64_t)(first + g) * 4096, 4096 * 8);
            double2 pv[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) pv[q] = ld_sc1(rg, (int64_t)(2 * (tid + 256 * q)) * 8);
#pragma unroll
            for (int q = 0; q < 8; ++q) { v[q].x += pv[q].x; v[q].y += pv[q].y; }
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = 2 * (tid + 256 * q), r = e >> 6, cl = e & 63;
            if (tflags) st_sc1(rC, ((int64_t)r * ld + cl) * 8, v[q]);
            else *reinterpret_cast<double2*>(S + (r0 + r) * ld + c0 + cl) = v[q];
        }
    }
    if (tflags) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_store(tflags + tk[7], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// syrk_body_wide: the same quarter task inside k_panel (512 threads, one workgroup per CU, its LDS
// free): all eight waves compute (wave w: rows 16 (w >> 1), columns 32 (w & 1) of the quarter, two
// 16x16 MFMA tiles), each source column's whole K = 128 panel of A and B (128 KB) is staged in LDS
// with one round of loads (16 x 16 B per thread in flight) instead of 32-deep slices, and the next
// source's panel is loaded into registers while the current one is multiplied.  Same sums in the
// same order per output element as syrk_body (k ascending within a source, sources ascending).
constexpr int LDW = 130;  // LDS row stride of a 128-deep panel (16-B aligned rows)
constexpr size_t SYRKW_LDS = sizeof(double) * 2 * 64 * LDW + 16;
__device__ __forceinline__ void syrk_body_wide(double* __restrict__ S, int64_t ld, const int32_t* __restrict__ tk,
                                               const int32_t* __restrict__ src, double* __restrict__ P,
                                               const int32_t* __restrict__ comb, unsigned* __restrict__ cnt,
                                               unsigned* __restrict__ tflags, double* __restrict__ smem,
                                               uint64_t* __restrict__ tr = nullptr) {
    double (*As)[LDW] = reinterpret_cast<double (*)[LDW]>(smem);
    double (*Bs)[LDW] = reinterpret_cast<double (*)[LDW]>(smem + 64 * LDW);
    unsigned* last = reinterpret_cast<unsigned*>(smem + 128 * LDW);
    const int64_t bi = tk[0], bj = tk[1];
    const int qr = tk[2] >> 1, qc = tk[2] & 1, s0 = tk[3], slot = tk[5];
    const int ns = tk[4] - s0;
    const int32_t* ks_src = src + s0;
    const int64_t r0 = bi * CB + qr * 64, c0 = bj * CB + qc * 64;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int lr = lane & 15, lk = lane >> 4;
    const int wr = (wave >> 1) * 16, wc = (wave & 1) * 32;
    double* Cp = slot < 0 ? S + (r0 + wr + lk) * ld + c0 + wc + lr : P + (int64_t)slot * 4096 + (wr + lk) * 64 + wc + lr;
    const int64_t ldc = slot < 0 ? ld : 64;
    dbl4 acc[2];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[b][r] = slot < 0 ? Cp[(4 * r) * ldc + b * 16] : 0.0;
    // loader mapping: wave w loads rows w, w + 8, .. of A and of B, lane l columns 2l, 2l + 1: one wave
    // instruction reads one whole 1 KB row (8 cache lines), 16 of them in flight per lane
    const double* ga = S + (r0 + wave) * ld + 2 * lane;
    const double* gb = S + (c0 + wave) * ld + 2 * lane;
    double2 pa[8], pb[8];
    auto load = [&](int k) {
        const int64_t kc = (int64_t)ks_src[k] * CB;
#pragma unroll
        for (int h = 0; h < 8; ++h) {
            pa[h] = *reinterpret_cast<const double2*>(ga + (int64_t)(8 * h) * ld + kc);
            pb[h] = *reinterpret_cast<const double2*>(gb + (int64_t)(8 * h) * ld + kc);
        }
    };
    load(0);
    for (int k = 0; k < ns; ++k) {
        if (k > 0) __syncthreads();  // the previous source's panels are consumed
#pragma unroll
        for (int h = 0; h < 8; ++h) {  // (component stores: a double2 struct copy kept the arrays in scratch)
            As[wave + 8 * h][2 * lane] = pa[h].x; As[wave + 8 * h][2 * lane + 1] = pa[h].y;
            Bs[wave + 8 * h][2 * lane] = pb[h].x; Bs[wave + 8 * h][2 * lane + 1] = pb[h].y;
        }
        __syncthreads();
        if (tr && tid == 0 && k == 0) tr[4] = wall_clock64();  // FBA_PANEL_TRACE: first panels in LDS
        if (k + 1 < ns) load(k + 1);  // the next source in flight while this one is multiplied
#pragma unroll
        for (int kb = 0; kb < CB; kb += 32) {  // operands of 8 k-steps read ahead of their MFMAs
            double av[8], b0[8], b1[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                av[q] = -As[wr + lr][kb + 4 * q + lk];
                b0[q] = Bs[wc + lr][kb + 4 * q + lk];
                b1[q] = Bs[wc + 16 + lr][kb + 4 * q + lk];
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                acc[0] = mfma(av[q], b0[q], acc[0]);
                acc[1] = mfma(av[q], b1[q], acc[1]);
            }
        }
    }
    const __amdgpu_buffer_rsrc_t rC = block_rsrc(S + r0 * ld + c0, ((int64_t)63 * ld + 64) * 8);
    if (tr && tid == 0) tr[5] = wall_clock64();  // products done (wave 0)
    if (slot < 0) {
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (tflags)
                    st_sc1(rC, ((int64_t)(wr + lk + 4 * r) * ld + wc + lr + b * 16) * 8, acc[b][r]);
                else
                    Cp[(4 * r) * ldc + b * 16] = acc[b][r];
            }
        if (tflags) {  // publish the quarter
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) __hip_atomic_store(tflags + tk[7], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    // split target (as syrk_body): the partial to scratch write-through, the last group adds the groups
    // in slot order
    {
        const __amdgpu_buffer_rsrc_t rP = block_rsrc(P + (int64_t)slot * 4096, 4096 * 8);
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                st_sc1(rP, (int64_t)((wr + lk + 4 * r) * 64 + wc + lr + b * 16) * 8, acc[b][r]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int32_t* cb = comb + Sched::COMB_REC * tk[6];
    if (tid == 0)
        *last = __hip_atomic_fetch_add(cnt + tk[6], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(cb[4] - 1);
    __syncthreads();
    if (!*last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const int first = cb[3], n = cb[4];
    double2 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int e = 2 * (tid + 512 * q), r = e >> 6, cl = e & 63;
        v[q] = *reinterpret_cast<const double2*>(S + (r0 + r) * ld + c0 + cl);
    }
    for (int g = 0; g < n; ++g) {
        const __amdgpu_buffer_rsrc_t rg = block_rsrc(P + (int64_t)(first + g) * 4096, 4096 * 8);
        double2 pv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) pv[q] = ld_sc1(rg, (int64_t)(2 * (tid + 512 * q)) * 8);
#pragma unroll
        for (int q = 0; q < 4; ++q) { v[q].x += pv[q].x; v[q].y += pv[q].y; }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int e = 2 * (tid + 512 * q), r = e >> 6, cl = e & 63;
        if (tflags) st_sc1(rC, ((int64_t)r * ld + cl) * 8, v[q]);
        else *reinterpret_cast<double2*>(S + (r0 + r) * ld + c0 + cl) = v[q];
    }
    if (tflags) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_store(tflags + tk[7], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ __launch_bounds__(256) void k_syrk_multi(double* __restrict__ S, int64_t ld, const int32_t* __restrict__ tasks,
                                                    const int32_t* __restrict__ src, double* __restrict__ P,
                                                    const int32_t* __restrict__ comb, unsigned* __restrict__ cnt) {
    __shared__ __attribute__((aligned(16))) double sm[128 * LDK + 2];
    syrk_body(S, ld, tasks + Sched::SYRK_REC * blockIdx.x, src, P, comb, cnt, nullptr, sm);
}

// ------------------------------------------------------------------------------------------------
// border combine (inner constraints): RHS rows n_pad + 0 (y) and n_pad + 1..7 (Z), length n
// ------------------------------------------------------------------------------------------------
// k_border_gram: the Gram matrix of the 15 forward-solved RHS rows [y | A (7) | B (7)]: GRAM_SEG
// workgroups, each a contiguous range of 128-column tiles staged through LDS, the 120 entries (a <= b)
// of its range into gpart[seg][120]
constexpr int GRAM_SEG = 16;

__global__ __launch_bounds__(256) void k_border_gram(const double* __restrict__ S, int64_t ld, int64_t n_pad,
                                                     double* __restrict__ gpart) {
    __shared__ double R[15][CB + 1];
    __shared__ double half[2][120];
    const int tid = threadIdx.x, seg = blockIdx.x;
    const int64_t nt = n_pad / CB, t0 = nt * seg / GRAM_SEG, t1 = nt * (seg + 1) / GRAM_SEG;
    const int e = tid % 120, h = tid / 120;  // threads 0..239: entry e, half h of the 128 columns
    int a = 0, rem = e;
    while (rem >= 15 - a) { rem -= 15 - a; ++a; }
    const int b = a + rem;
    double v = 0.0;
    for (int64_t t = t0; t < t1; ++t) {
        __syncthreads();
        double x[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int i = tid + 256 * q;
            x[q] = i < 15 * CB ? S[(n_pad + i / CB) * ld + t * CB + i % CB] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int i = tid + 256 * q;
            if (i < 15 * CB) R[i / CB][i % CB] = x[q];
        }
        __syncthreads();
        if (h < 2)
            for (int k = 64 * h; k < 64 * h + 64; ++k) v += R[a][k] * R[b][k];
    }
    if (h < 2) half[h][e] = v;
    __syncthreads();
    if (tid < 120) gpart[(int64_t)seg * 120 + tid] = half[0][tid] + half[1][tid];
}

// k_border_combine: every workgroup adds the Gram segments (fixed order), solves
// [[A'A - I, A'B], [B'A, B'B]] [z; k] = -[A'y; B'y] (14x14, partial pivoting, wave 0 alone) and forms
// u = y + A z + B k on its 256 entries of the RHS row (derivation in fba_kernels.hip, border section)
// gblk != nullptr: the Gram comes as nblk per-column-block 16x16 partials (k_chol_flow's RHS panel
// halves, row-major, rows/columns 15 zero), added in block order instead of the GRAM_SEG segments
// the 14 coefficients into coef[] (LDS, 256 threads; g: 15 x 15 LDS scratch); ends with a barrier
// bsc (subtree split): the B rows were forward-solved unscaled; their Gram entries take the factors
// sqrt(W_d) here (rows / columns 8..14) and so do the B coefficients handed on, so u = y + A z + B (bsc k)
// is the one-GPU combine's y + A z + (B bsc) k
__device__ __forceinline__ void border_combine_body(const double* __restrict__ gpart, const double* __restrict__ gblk,
                                                    int nblk, double (*g)[15], double* coef,
                                                    const double* __restrict__ bsc = nullptr) {
    const int tid = threadIdx.x;
    if (tid < 120) {
        int a = 0, rem = tid;
        while (rem >= 15 - a) { rem -= 15 - a; ++a; }
        const int b = a + rem;
        double v = 0.0;
        if (gblk) {
            for (int q = 0; q < nblk; q += 32) {  // 32 loads in flight, the same running sum
                double x[32];
#pragma unroll
                for (int u = 0; u < 32; ++u) x[u] = q + u < nblk ? gblk[(int64_t)(q + u) * 256 + a * 16 + b] : 0.0;
#pragma unroll
                for (int u = 0; u < 32; ++u)
                    if (q + u < nblk) v += x[u];
            }
        } else {
            double x[GRAM_SEG];
#pragma unroll
            for (int q = 0; q < GRAM_SEG; ++q) x[q] = gpart[q * 120 + tid];
#pragma unroll
            for (int q = 0; q < GRAM_SEG; ++q) v += x[q];
        }
        if (bsc) v *= (a >= 8 ? bsc[a - 8] : 1.0) * (b >= 8 ? bsc[b - 8] : 1.0);
        g[a][b] = g[b][a] = v;
    }
    __syncthreads();
    if (tid < 64) {
        // wave 0: lane r < 14 holds row r of the augmented H = [H | rhs] in registers.  The pivot search
        // is a DPP max-reduction over the 16-lane row (no LDS round trips), the pivot row and row col are
        // broadcast with v_readlane from their (uniform) lanes, so a step is a few dozen VALU
        // instructions.  The arithmetic and its order are those of the plain row-by-row elimination
        // and back substitution.
        double h[15];
        if (tid < 14) {
#pragma unroll
            for (int q = 0; q < 14; ++q) h[q] = g[1 + tid][1 + q] - ((tid == q && tid < 7) ? 1.0 : 0.0);
            h[14] = -g[1 + tid][0];
        } else {
#pragma unroll
            for (int q = 0; q < 15; ++q) h[q] = 0.0;
        }
        // v = max |candidate|, ties to the lower row; p its row (lanes outside [col, 14) seed p = col,
        // so an all-NaN column keeps the pivot at col, as the serial search does)
        auto take = [](double& v, int& p, double ov, int op) {
            if (ov > v || (ov == v && op < p)) { v = ov; p = op; }
        };
#pragma unroll
        for (int col = 0; col < 14; ++col) {
            double v = (tid >= col && tid < 14) ? fabs(h[col]) : -1.0;
            int p = (tid >= col && tid < 14) ? tid : col;
            take(v, p, dpp_f64<0xB1>(v), __builtin_amdgcn_mov_dpp(p, 0xB1, 0xF, 0xF, false));    // quad_perm [1,0,3,2]
            take(v, p, dpp_f64<0x4E>(v), __builtin_amdgcn_mov_dpp(p, 0x4E, 0xF, 0xF, false));    // quad_perm [2,3,0,1]
            take(v, p, dpp_f64<0x141>(v), __builtin_amdgcn_mov_dpp(p, 0x141, 0xF, 0xF, false));  // row_half_mirror
            take(v, p, dpp_f64<0x140>(v), __builtin_amdgcn_mov_dpp(p, 0x140, 0xF, 0xF, false));  // row_mirror
            p = __builtin_amdgcn_readfirstlane(p);
            double piv[15];
#pragma unroll
            for (int q = col; q < 15; ++q) {
                const double hp = readlane_d(h[q], p), hc = readlane_d(h[q], col);
                if (tid == p) h[q] = hc;     // row swap (a no-op when p == col)
                if (tid == col) h[q] = hp;
                piv[q] = hp;                 // the pivot row after the swap
            }
            if (tid > col && tid < 14) {
                const double f = h[col] / piv[col];
#pragma unroll
                for (int q = col; q < 15; ++q) h[q] -= f * piv[q];
            }
        }
        // back substitution, rows 13..0, each row's sum in ascending column order
        double c[14];
#pragma unroll
        for (int r = 13; r >= 0; --r) {
            double v = h[14];
#pragma unroll
            for (int q = r + 1; q < 14; ++q) v -= h[q] * c[q];
            c[r] = readlane_d(v / h[r], r);
        }
        if (tid < 14) {
            double mine = c[0];
#pragma unroll
            for (int q = 1; q < 14; ++q) mine = (tid == q) ? c[q] : mine;
            coef[tid] = (bsc && tid >= 7) ? mine * bsc[tid - 7] : mine;
        }
    }
    __syncthreads();
}

__global__ __launch_bounds__(256) void k_border_combine(double* __restrict__ S, int64_t ld, int64_t n_pad,
                                                        const double* __restrict__ gpart, double* __restrict__ coef_out,
                                                        const double* __restrict__ gblk = nullptr, int nblk = 0) {
    __shared__ double g[15][15];
    __shared__ double coef[14];
    const int tid = threadIdx.x;
    border_combine_body(gpart, gblk, nblk, g, coef);
    if (coef_out) {  // one workgroup: the 14 coefficients only (k_bwd_flow applies them)
        if (tid < 14) coef_out[tid] = coef[tid];
        return;
    }
    const int64_t i = (int64_t)blockIdx.x * 256 + tid;
    if (i < n_pad) {
        double* yw = S + n_pad * ld;
        double v = yw[i];
#pragma unroll
        for (int m = 0; m < 14; ++m) v += S[(n_pad + 1 + m) * ld + i] * coef[m];
        yw[i] = v;
    }
}

constexpr size_t TRTRI_LDS = sizeof(double) * (CB * LDA + 4 * IB * 17 + IB * LDA);  // X, per-wave staging, L row block

// ------------------------------------------------------------------------------------------------
// k_trtri128: inverse of the 128x128 diagonal blocks (the listed columns, or all; one workgroup per
// block, after the factorisation): block forward substitution on the 8x8 grid of 16x16 tiles,
// X_ii = D_i, X_ij = -D_i sum_{k=j}^{i-1} L_ik X_kj, on v_mfma_f64_16x16x4_f64.
// ------------------------------------------------------------------------------------------------
// trtri_body: threads 0..255 of the workgroup invert block kb; threads 256.. (a k_panel workgroup
// has 512) only take part in the barriers
__device__ __forceinline__ void trtri_body(const double* __restrict__ S, int64_t ld, int kb,
                                           const double* __restrict__ dinv, double* __restrict__ linv,
                                           double* __restrict__ smem) {
    double* X = smem;                   // [128][LDA]
    double* Y = smem + CB * LDA;        // [4 waves][16][17]
    const int tid = threadIdx.x, wave = (tid & 255) >> 6, lane = tid & 63;
    const bool worker = tid < 256;
    const int lr = lane & 15, lk = lane >> 4;
    const double* L = S + (int64_t)kb * CB * ld + (int64_t)kb * CB;
    const double* Dk = dinv + (int64_t)kb * (CB / IB) * (IB * IB);
    // row block i of L (16 x 128) staged in LDS for step i; the next one is loaded into registers
    // while step i computes (the row reads were the latency of every step)
    double* Lr = Y + 4 * IB * 17;       // [16][LDA]
    double lpre[8];
    if (worker) {
        for (int idx = tid; idx < CB * CB; idx += 256) {
            const int r = idx >> 7, c = idx & 127;
            X[r * LDA + c] = ((r >> 4) == (c >> 4)) ? Dk[(r >> 4) * IB * IB + (r & 15) * IB + (c & 15)] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int idx = tid + 256 * q;
            lpre[q] = L[(int64_t)(IB + (idx >> 7)) * ld + (idx & 127)];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int idx = tid + 256 * q;
            Lr[(idx >> 7) * LDA + (idx & 127)] = lpre[q];
        }
    }
    __syncthreads();
    double* Yw = Y + wave * IB * 17;
    for (int i = 1; i < CB / IB; ++i) {
        if (worker) {
            if (i + 1 < CB / IB) {
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int idx = tid + 256 * q;
                    lpre[q] = L[(int64_t)(IB * (i + 1) + (idx >> 7)) * ld + (idx & 127)];
                }
            }
            for (int j = wave; j < i; j += 4) {
                dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
                for (int k = j; k < i; ++k) {
#pragma unroll
                    for (int kk = 0; kk < IB; kk += 4) {
                        const double av = Lr[lr * LDA + IB * k + kk + lk];
                        const double bv = X[(IB * k + kk + lk) * LDA + IB * j + lr];
                        acc = mfma(av, bv, acc);
                    }
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) Yw[(lk + 4 * r) * 17 + lr] = acc[r];
                __builtin_amdgcn_s_waitcnt(0xC07F);
                __builtin_amdgcn_wave_barrier();
                dbl4 out = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int kk = 0; kk < IB; kk += 4) {
                    const double av = -X[(IB * i + lr) * LDA + IB * i + kk + lk];  // D_i, the diagonal tile of X
                    const double bv = Yw[(kk + lk) * 17 + lr];
                    out = mfma(av, bv, out);
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) X[(IB * i + lk + 4 * r) * LDA + IB * j + lr] = out[r];
                __builtin_amdgcn_s_waitcnt(0xC07F);
                __builtin_amdgcn_wave_barrier();
            }
        }
        __syncthreads();
        if (i + 1 < CB / IB) {
            if (worker)
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int idx = tid + 256 * q;
                    Lr[(idx >> 7) * LDA + (idx & 127)] = lpre[q];
                }
            __syncthreads();
        }
    }
    if (worker) {
        double* out = linv + (int64_t)kb * CB * CB;
        for (int idx = tid; idx < CB * CB; idx += 256) out[idx] = X[(idx >> 7) * LDA + (idx & 127)];
    }
}

__global__ __launch_bounds__(256) void k_trtri128(const double* __restrict__ S, int64_t ld, const int32_t* __restrict__ cols,
                                                  const double* __restrict__ dinv, double* __restrict__ linv) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    trtri_body(S, ld, cols ? cols[blockIdx.x] : (int)blockIdx.x, dinv, linv, smem);
}

// k_panel: one level's diagonal factorisations and panel solves in ONE launch: workgroups
// 0 .. ncol-1 factor the level's diagonal blocks (potrf_body) and publish them, the next ntrsm solve
// the panel halves (trsm_body) as soon as their column's factor is published, and the last nprev
// invert the diagonal blocks of the PREVIOUS level (trtri_body; final since the last launch) for the
// backward solve, off the critical path.  Every workgroup of the launch is resident at once (<= 8 +
// 2 * panel blocks + 8 workgroups, one per CU), so the waits end.
constexpr size_t PANEL_LDS_ = TRSM_LDS > TRTRI_LDS ? TRSM_LDS : TRTRI_LDS;
constexpr size_t PANEL_LDS = PANEL_LDS_ > SYRKW_LDS ? PANEL_LDS_ : SYRKW_LDS;

__global__ __launch_bounds__(POTRF_THREADS) void k_panel(double* __restrict__ S, int64_t ld, const int32_t* __restrict__ cols,
                                                         int ncol, const int32_t* __restrict__ trsm, int ntrsm,
                                                         const int32_t* __restrict__ prev, int nprev,
                                                         double* __restrict__ dinv,
                                                         double* __restrict__ linv, double* __restrict__ scal,
                                                         unsigned* __restrict__ flags, int progressive,
                                                         const int32_t* __restrict__ tasks, int ntask, int ndiag,
                                                         int npanel, const int32_t* __restrict__ src,
                                                         double* __restrict__ P, const int32_t* __restrict__ comb,
                                                         unsigned* __restrict__ cnt, unsigned* __restrict__ tflags,
                                                         const int32_t* __restrict__ wstart,
                                                         const int32_t* __restrict__ wlist,
                                                         uint64_t* __restrict__ trace) {
    // workgroup order (every wait points to a lower index, so in-order dispatch always progresses):
    // [the previous level's updates of this level's diagonal blocks][potrf][its updates of this level's
    // panel blocks][panel solves][inverses of the previous level's blocks][its updates of later levels'
    // blocks, which nothing in this launch waits for]
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int b = blockIdx.x;
    const int e1 = ndiag, e2 = e1 + ncol, e3 = e2 + npanel, e4 = e3 + ntrsm, e5 = e4 + nprev;
    // FBA_PANEL_TRACE: [start, after the waits, end, role, phase stamps] per workgroup (100 MHz wall clock)
    // (PTRACE_WG slots per level: a larger grid leaves its extra workgroups untraced)
    uint64_t* tr = (trace && b < PTRACE_WG) ? trace + 8 * (int64_t)b : nullptr;
    if (tr && threadIdx.x == 0) tr[0] = wall_clock64();
    int role;
    if (b < e1) {
        role = 0;
        if (tr && threadIdx.x == 0) {  // FBA_PANEL_TRACE: sources, split group
            const int32_t* tk = tasks + Sched::SYRK_REC * b;
            tr[1] = (uint64_t)(tk[4] - tk[3]) | (tk[5] >= 0 ? 0x100u : 0u);
        }
        syrk_body_wide(S, ld, tasks + Sched::SYRK_REC * b, src, P, comb, cnt, tflags, smem, tr);
    } else if (b < e2) {
        role = 1;
        const int c = b - e1;
        if (ntask > 0) wait_list(wlist + wstart[c], wstart[c + 1] - wstart[c], tflags, scal);
        if (tr && threadIdx.x == 0) tr[1] = wall_clock64();
        potrf_body<false>(S, ld, cols[c], dinv, scal, nullptr, flags + cols[c], smem);
    } else if (b < e3) {
        role = 2;
        syrk_body_wide(S, ld, tasks + Sched::SYRK_REC * (b - ncol), src, P, comb, cnt, tflags, smem);
    } else if (b < e4) {
        role = 3;
        const int t = b - e3;
        if (ntask > 0) wait_list(wlist + wstart[ncol + t], wstart[ncol + t + 1] - wstart[ncol + t], tflags, scal);
        const int32_t* rec = trsm + 2 * t;
        trsm_body(S, ld, rec, dinv, flags + rec[0], scal, smem, progressive != 0, tr);
    } else if (b < e5) {
        role = 4;
        trtri_body(S, ld, prev[b - e4], dinv, linv, smem);
    } else {
        role = 5;
        syrk_body_wide(S, ld, tasks + Sched::SYRK_REC * (b - e5 + ndiag + npanel), src, P, comb, cnt, tflags, smem);
    }
    if (tr) {  // uniform: the trace pointer is a kernel argument
        __syncthreads();
        if (threadIdx.x == 0) {
            tr[2] = wall_clock64();
            tr[3] = (uint64_t)role;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// k_chol_flow: the whole block factorisation as ONE persistent launch (schedule: fba_order.cpp
// build_flow).  One 512-thread workgroup per record; every wait points to an earlier record.
// ------------------------------------------------------------------------------------------------

// trsm_flow_body (k_chol_flow role 1): one 64-row half of panel block (r, k), X = A L_kk^-T, RIGHT-looking
// with each solving wave's 16 rows of A in registers: as block column t of L_kk arrives (waves 4-7
// load it into LDS as k's potrf publishes it, as in trsm_body), X_t = A_t D_t', then A_s -= X_t L_st' for
// s > t -- so after the last column only X_7 = A_7 D_7' is left.  Every solved column block is stored
// write-through; its drain overlaps the next step, after which the last of the four solving waves
// raises the progress flag (prog = column blocks published).
constexpr size_t TRSMF_LDS = sizeof(double) * (4 * IB * 17 + (TRSM_NT + CB / IB) * IB * 17) + 16 * sizeof(int);
__device__ __forceinline__ void trsm_flow_body(double* __restrict__ S, int64_t ld, const int32_t* __restrict__ rec,
                                               const double* __restrict__ dinv, const unsigned* __restrict__ flag,
                                               double* __restrict__ scal, double* __restrict__ smem,
                                               uint64_t* __restrict__ tr, unsigned* __restrict__ prog,
                                               double* __restrict__ gram) {
    double* T = smem;                       // [4][IB][17]    per-wave transposes
    double* Lt = T + 4 * IB * 17;           // [28][IB][17]   L_st, p = s(s-1)/2 + t
    double* Dt = Lt + TRSM_NT * IB * 17;    // [8][IB][17]    D_s
    int* s_col = reinterpret_cast<int*>(Dt + (CB / IB) * IB * 17);  // [8] column t in LDS
    int* s_cnt = s_col + CB / IB;                                    // [8] solving waves done with step t
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int lr = lane & 15, lk = lane >> 4;
    const bool worker = tid < 256;
    const int64_t k0 = (int64_t)rec[0] * CB;
    const int rh = rec[1];
    const int64_t rbase = (int64_t)(rh >> 1) * CB + (rh & 1) * 64 + (wave & 3) * IB;
    const double* L = S + k0 * ld + k0;
    const double* Dk = dinv + (k0 / CB) * (CB / IB) * (IB * IB);
    if (tid < 2 * (CB / IB)) s_col[tid] = 0;
    const __amdgpu_buffer_rsrc_t rX = block_rsrc(S + rbase * ld + k0, ((int64_t)(IB - 1) * ld + CB) * 8);
    dbl4 acc[CB / IB];
    if (worker)  // this wave's 16 rows of A, MFMA output layout: acc[t][r] = A[lk + 4 r][16 t + lr]
#pragma unroll
        for (int t = 0; t < CB / IB; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                acc[t][r] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                                           rX, (int)(((int64_t)(lk + 4 * r) * ld + IB * t + lr) * 8), 0, SC1));
    __syncthreads();  // the flags are zero
    if (!worker) {
        // the four loader waves share every column (a single wave reading freshly written-through
        // data gets only a few GB/s): wave 4 + v takes items v, v + 4, .. of the column's (8 - t) * 128
        // double2, each raising the column's LDS count once its share is in
        const __amdgpu_buffer_rsrc_t rL = block_rsrc(L, ((int64_t)(CB - 1) * ld + CB) * 8);
        const __amdgpu_buffer_rsrc_t rD = block_rsrc(Dk, (CB / IB) * IB * IB * 8);
        const int v4 = wave - 4;
        for (int t = 0; t < CB / IB; ++t) {
            unsigned spins = 0;
            while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)(t + 1)) {
                __builtin_amdgcn_s_sleep(1);
                if (spin_expired(spins, scal)) break;  // (hand-off timeout or abort: reported by the host)
            }
            double2 v[4];
            double* dst[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {  // items (8 - t) * 128 double2, item i = 256 q + 64 v4 + lane
                const int i = 256 * q + 64 * v4 + lane, u = i >> 7, n = (i >> 3) & 15, kc = (i & 7) * 2;
                dst[q] = nullptr;
                if (u < CB / IB - 1 - t) {  // tile (r, t), r = t + 1 + u
                    const int r = t + 1 + u;
                    v[q] = ld_sc1(rL, ((int64_t)(r * IB + n) * ld + t * IB + kc) * 8);
                    dst[q] = Lt + ((r * (r - 1) / 2 + t) * IB + n) * 17 + kc;
                } else if (u == CB / IB - 1 - t) {  // D_t
                    v[q] = ld_sc1(rD, (int64_t)(t * IB * IB + n * IB + kc) * 8);
                    dst[q] = Dt + (t * IB + n) * 17 + kc;
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (dst[q]) {
                    dst[q][0] = v[q].x;
                    dst[q][1] = v[q].y;
                }
            __builtin_amdgcn_s_waitcnt(0xC07F);  // this wave's LDS writes done
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) __hip_atomic_fetch_add(s_col + t, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (tr && lane == 0 && v4 == 0) tr[8 + t] = wall_clock64();  // FBA_PANEL_TRACE: column t of L_kk in LDS
        }
        return;
    }
    double* Tw = T + wave * IB * 17;
    dbl4 gacc = dbl4{0.0, 0.0, 0.0, 0.0};  // the RHS half (gram != nullptr): the 16 x 16 Gram of wave 0's rows
    bool pending = false;  // column block t-1 stored, not yet signalled
    auto signal = [&](int done) {  // after this wave's drain: the last of the four raises the flag
        __builtin_amdgcn_wave_barrier();
        if (lane == 0 && __hip_atomic_fetch_add(s_cnt + done - 1, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP) == 3) {
            __hip_atomic_store(prog, (unsigned)done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (tr) tr[16 + done - 1] = wall_clock64();  // FBA_PANEL_TRACE: column block done-1 published
        }
    };
#pragma unroll
    for (int t = 0; t < CB / IB; ++t) {
        unsigned sp = 0;
        while (__hip_atomic_load(s_col + t, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < 4) {
            __builtin_amdgcn_s_sleep(1);
            if (spin_expired(sp, scal)) break;
        }
        // X_t = A_t D_t': A_t to the operand layout through Tw
#pragma unroll
        for (int r = 0; r < 4; ++r) Tw[(lk + 4 * r) * 17 + lr] = acc[t][r];
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        double av[4];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) av[kk] = Tw[lr * 17 + 4 * kk + lk];
        dbl4 x = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) x = mfma(av[kk], Dt[(t * IB + lr) * 17 + 4 * kk + lk], x);
#pragma unroll
        for (int r = 0; r < 4; ++r) Tw[(lk + 4 * r) * 17 + lr] = x[r];
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        double xa[4];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) xa[kk] = -Tw[lr * 17 + 4 * kk + lk];
        if (gram && wave == 0)  // the RHS rows (all in wave 0): G += X_t X_t'
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) gacc = mfma(xa[kk], xa[kk], gacc);
        if (t > 0 && pending) {  // column block t-1's stores drained during this step
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            signal(t);
        }
        {
            const int n = lane >> 2, m = 4 * (lane & 3);
            double2 v0, v1;
            v0.x = Tw[n * 17 + m];
            v0.y = Tw[n * 17 + m + 1];
            v1.x = Tw[n * 17 + m + 2];
            v1.y = Tw[n * 17 + m + 3];
            st_sc1(rX, ((int64_t)n * ld + IB * t + m) * 8, v0);
            st_sc1(rX, ((int64_t)n * ld + IB * t + m + 2) * 8, v1);
        }
        if (t == CB / IB - 1) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            signal(CB / IB);
            if (tr && tid == 0) tr[6] = wall_clock64();
        }
        // right-looking: A_s -= X_t L_st'
#pragma unroll
        for (int s = t + 1; s < CB / IB; ++s)
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
                acc[s] = mfma(xa[kk], Lt[((s * (s - 1) / 2 + t) * IB + lr) * 17 + 4 * kk + lk], acc[s]);
        // column block t published now if column t+1 has not arrived (the wave would only wait), else
        // drained during step t+1
        pending = true;
        if (t + 1 < CB / IB && __hip_atomic_load(s_col + t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 4) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            signal(t + 1);
            pending = false;
        }
    }
    if (gram && wave == 0)  // consumed by k_border_combine, the next launch
#pragma unroll
        for (int r = 0; r < 4; ++r) gram[(lk + 4 * r) * 16 + lr] = gacc[r];
}

// wait until every flag of a list is set, then a workgroup barrier; no acquire fence: every load of
// the handed-off bytes behind it is an sc1 load of sc1 stores (MI355X guide, hand-off table row 1)
__device__ __forceinline__ void wait_list_sc1(const int32_t* __restrict__ wl, int n, const unsigned* __restrict__ fl,
                                              double* __restrict__ scal) {
    if (n > 0 && threadIdx.x == 0)
        for (int q = 0; q < n; ++q) spin_ge(fl + wl[q], 1u, scal);
    __syncthreads();
}

// LDS of the diagonal-block role: the potrf's lower tiles, leaf inverses and counters, then a second
// 128 x 17 buffer for the fused source's published column blocks (the first is the leaf-inverse area,
// free until the potrf starts)
constexpr size_t FLOWF_LDS_FUSED = sizeof(double) * (POTRF_NT * IB * 17 + (CB / IB) * IB * 17) + 32 * sizeof(int) +
                                   sizeof(double) * CB * 17;
constexpr size_t FLOWF_LDS = FLOWF_LDS_FUSED;
static_assert(CB * 17 == (CB / IB) * IB * 17, "a column-block buffer is exactly the leaf-inverse area");

// fused_apply<SET>: C -= X X' on the tiles of SET, X = L(j, f) consumed column block by column block as
// the two panel-half records of (f, j) publish it (progress flags p0, p1): block t + 1's loads are issued
// before block t's update whenever it is already published, so the update (in registers, tiles spread
// over all eight waves) keeps pace with the panel solves.  SET 0/1: C from and back to the LDS block
// (smem, the potrf's tile layout); SET 2: from zero, to out (the helper's scratch partial).  X0, X1: two
// [128][17] LDS buffers; sy[31] a word.
template <int SET>
__device__ __forceinline__ void fused_apply(const __amdgpu_buffer_rsrc_t rX, int64_t ld, const unsigned* __restrict__ p0,
                                            const unsigned* __restrict__ p1, double* __restrict__ X0,
                                            double* __restrict__ X1, int* __restrict__ sy, double* __restrict__ smem,
                                            double* __restrict__ out, double* __restrict__ scal, uint64_t* __restrict__ tr) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int lr = lane & 15, lk = lane >> 4;
    double* Xb[2] = {X0, X1};
    auto published = [&]() {
        unsigned v = __hip_atomic_load(p0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (p1) v = std::min(v, __hip_atomic_load(p1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        return v;
    };
    // column block b (128 rows x 16) is loaded by ONE group of waves, b mod 3: waves 1-3 (six 16-B items
    // per lane), waves 4-5 or waves 6-7 (eight each), item i -> row i >> 3, columns 2 (i & 7), +1; wave 0
    // loads nothing and thread 0 reads the progress flags.  So every wave has at most one block's loads
    // in flight and the compiler's wait before storing a block into LDS waits for that block alone,
    // while the other groups' blocks (t + 1, t + 2) stay in flight across the barrier: three blocks in
    // flight, so a diagonal workgroup that starts behind its panel halves catches up at about a third
    // of an sc1 round trip per block (with two groups it took ~2 us per block, the loads' latency / 2)
    constexpr int NGRP = 3;
    const int grp = wave == 0 ? -1 : (wave < 4 ? 0 : (wave < 6 ? 1 : 2));
    const int gl = grp == 0 ? tid - 64 : (grp == 1 ? tid - 256 : tid - 384);
    constexpr int GM = 8;  // items per lane (group 0: 6)
    double2 xl[GM];
    auto issue = [&](int b) {
        if (grp != b % NGRP) return;
#pragma unroll
        for (int m = 0; m < GM; ++m) {
            const int i = gl + (grp == 0 ? 192 : 128) * m;
            if ((grp != 0 || m < 6) && i < 1024)
                xl[m] = ld_sc1(rX, ((int64_t)(i >> 3) * ld + IB * b + 2 * (i & 7)) * 8);
        }
    };
    auto store = [&](int b, double* X) {
        if (grp != b % NGRP) return;
#pragma unroll
        for (int m = 0; m < GM; ++m) {
            const int i = gl + (grp == 0 ? 192 : 128) * m;
            if ((grp != 0 || m < 6) && i < 1024) {
                X[(i >> 3) * 17 + 2 * (i & 7)] = xl[m].x;
                X[(i >> 3) * 17 + 2 * (i & 7) + 1] = xl[m].y;
            }
        }
    };
    // thread 0: the progress values last read (issued after a barrier, their min taken at the next, so
    // wave 0 does not wait for the loads before its update)
    unsigned fv, fv0 = 0, fv1 = ~0u;
    auto wait_pub = [&](int b) {  // column block b published (thread 0 polls), then the barrier
        if (tid == 0) {
            unsigned spins = 0;
            while ((fv = published()) <= (unsigned)b) {
                __builtin_amdgcn_s_sleep(1);
                if (spin_expired(spins, scal)) break;
            }
            fv0 = fv;
            fv1 = ~0u;
        }
        __syncthreads();
    };
    int issued = 0;          // blocks [0, issued) issued (uniform)
    wait_pub(0);             // (its barrier also completes the C_jj load)
    constexpr int NS = fset_count(SET), NT = (NS + POTRF_NW - 1) / POTRF_NW;  // tiles of the set, per wave at most
    int ta[NT], tb[NT];
    dbl4 c[NT];  // this wave's tiles wave + 8 i of the set, in registers until the last block
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        fset_tile(SET, wave + POTRF_NW * i, ta[i], tb[i]);
        if (wave + POTRF_NW * i < NS)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                c[i][r] = SET == 2 ? 0.0 : smem[(ta[i] * (ta[i] + 1) / 2 + tb[i]) * IB * 17 + (lk + 4 * r) * 17 + lr];
    }
#pragma unroll
    for (int t = 0; t < CB / IB; ++t) {
        double* X = Xb[t & 1];
        if (issued <= t) {  // not in flight yet: wait for it
            wait_pub(t);
            issue(t);
            issued = t + 1;
        }
        store(t, X);
        if (tr && tid == (t % NGRP == 0 ? 64 : (t % NGRP == 1 ? 256 : 384)))
            tr[40 + t] = wall_clock64();  // FBA_PANEL_TRACE: group's share stored
        // (block t + 1 not in flight yet: read the flags now rather than use the values read during the
        // last update, which would issue it one update later)
        if (tid == 0) sy[31] = (int)(issued == t + 1 && t + 1 < CB / IB ? published() : std::min(fv0, fv1));
        __syncthreads();  // block t in LDS; the other buffer's readers (block t-1) are done
        if (tr && tid == 0) tr[8 + t] = wall_clock64();  // FBA_PANEL_TRACE: block t in LDS
        const int pub = sy[31];
        const bool pre = issued > t + 1 || (t + 1 < CB / IB && pub > t + 1);
        // blocks t+1, t+2 (the groups idle since they stored t-2, t-1) and t+3 (this block's group) in
        // flight during this update, as far as published
#pragma unroll
        for (int d = 1; d <= NGRP; ++d)
            if (issued == t + d && t + d < CB / IB && pub > t + d) {
                issue(t + d);
                issued = t + d + 1;
            }
        if (tid == 0) {  // consumed before the next barrier, after this update
            fv0 = __hip_atomic_load(p0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            fv1 = p1 ? __hip_atomic_load(p1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ~0u;
        }
        // C(a, b) -= X_t(a) X_t(b)' on this wave's tiles of the set
        double xa[NT][4], yb[NT][4];
#pragma unroll
        for (int i = 0; i < NT; ++i)
            if (wave + POTRF_NW * i < NS) {
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    xa[i][kk] = -X[(IB * ta[i] + lr) * 17 + 4 * kk + lk];
                    yb[i][kk] = X[(IB * tb[i] + lr) * 17 + 4 * kk + lk];
                }
            }
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int i = 0; i < NT; ++i)
                if (wave + POTRF_NW * i < NS) c[i] = mfma(xa[i][kk], yb[i][kk], c[i]);
        if (t == CB / IB - 1)
#pragma unroll
            for (int i = 0; i < NT; ++i)
                if (wave + POTRF_NW * i < NS) {
                    if (SET == 2)  // the helper: its tiles to the scratch partial, 16 x 16 row-major each
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            __hip_atomic_store(out + (wave + POTRF_NW * i) * IB * IB + (lk + 4 * r) * IB + lr, c[i][r],
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    else
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            smem[(ta[i] * (ta[i] + 1) / 2 + tb[i]) * IB * 17 + (lk + 4 * r) * 17 + lr] = c[i][r];
                }
        if (tr && tid == 0) tr[16 + t] = wall_clock64() | (pre ? (1ull << 63) : 0);  // block t applied
    }
}

// diag_body (role 0): diagonal block j.  C_jj (its final in-place writers done) is loaded into LDS; with
// a fused source f (rec[2] >= 0) C_jj -= X X', X = L(j, f), as the panel halves of (f, j) publish X
// (fused_apply: all tiles, or with a split helper, rec[9] >= 0, those of tile columns < FLOW_CSPLIT);
// then the late partials (the other sources of f's level, scratch quarters, slot order); then the potrf
// on the LDS block, whose bulk waves add the helper's partial (scratch slot rec[10], flag rec[9]).
__device__ __forceinline__ void diag_body(double* __restrict__ S, int64_t ld, const int32_t* __restrict__ rec,
                                          const int32_t* __restrict__ lists, double* __restrict__ dinv,
                                          double* __restrict__ scal, unsigned* __restrict__ colflags,
                                          unsigned* __restrict__ fl, const double* __restrict__ P,
                                          double* __restrict__ smem, uint64_t* __restrict__ tr) {
    const int j = rec[1], f = rec[2];
    wait_list_sc1(lists + rec[3], rec[4], fl, scal);  // the final in-place writers of C_jj's quarters
    if (tr && threadIdx.x == 0) tr[1] = wall_clock64();
    if (f < 0 && rec[6] == 0) {
        potrf_body<false>(S, ld, j, dinv, scal, nullptr, colflags + j, smem, tr ? tr + 16 : nullptr);
        return;
    }
#define AT(r, c) smem[(((r) >> 4) * (((r) >> 4) + 1) / 2 + ((c) >> 4)) * (IB * 17) + ((r) & 15) * 17 + ((c) & 15)]
    const int tid = threadIdx.x;
    const int64_t k0 = (int64_t)j * CB;
    double* Dall = smem + POTRF_NT * IB * 17;
    int* sy = reinterpret_cast<int*>(Dall + (CB / IB) * IB * 17);
    double* Xb[2] = {Dall, reinterpret_cast<double*>(sy + 32)};  // [128][17] each
    {   // C_jj's lower tiles into LDS
        const __amdgpu_buffer_rsrc_t rC = block_rsrc(S + k0 * ld + k0, ((int64_t)(CB - 1) * ld + CB) * 8);
        constexpr int NQ = POTRF_NT * 128 / POTRF_THREADS;  // 9
        double2 v[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int i = tid + POTRF_THREADS * q, p = i >> 7, n = (i >> 3) & 15, m = (i & 7) * 2;
            int ti = 0, pp = p;
            while (pp > ti) { pp -= ti + 1; ++ti; }
            v[q] = ld_sc1(rC, ((int64_t)(ti * IB + n) * ld + pp * IB + m) * 8);
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int i = tid + POTRF_THREADS * q, p = i >> 7, n = (i >> 3) & 15, m = (i & 7) * 2;
            smem[p * IB * 17 + n * 17 + m] = v[q].x;
            smem[p * IB * 17 + n * 17 + m + 1] = v[q].y;
        }
    }
    if (f >= 0) {
        const int64_t f0 = (int64_t)f * CB;
        const __amdgpu_buffer_rsrc_t rX = block_rsrc(S + k0 * ld + f0, ((int64_t)(CB - 1) * ld + CB) * 8);
        const unsigned* p0 = fl + rec[7];
        const unsigned* p1 = rec[8] >= 0 ? fl + rec[8] : nullptr;
        if (rec[9] >= 0)  // split: the tiles of tile columns >= FLOW_CSPLIT come from the helper record
            fused_apply<1>(rX, ld, p0, p1, Xb[0], Xb[1], sy, smem, nullptr, scal, tr);
        else
            fused_apply<0>(rX, ld, p0, p1, Xb[0], Xb[1], sy, smem, nullptr, scal, tr);
    }
    if (tr && threadIdx.x == 0) tr[4] = wall_clock64();
    // late partials: the other sources of f's level, 64x64 row-major scratch quarters, added in slot
    // order; every flag checked first, then up to four partials' loads in flight together
    if (rec[6] > 0) {
        __syncthreads();
        if (tid == 0)
            for (int e = 0; e < rec[6]; ++e) spin_ge(fl + lists[rec[5] + 3 * e + 2], 1u, scal);
        __syncthreads();
    }
    for (int e0 = 0; e0 < rec[6]; e0 += 4) {
        const int ne = rec[6] - e0 < 4 ? rec[6] - e0 : 4;
        double2 v[4][4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (e < ne) {
                const __amdgpu_buffer_rsrc_t rp = block_rsrc(P + (int64_t)lists[rec[5] + 3 * (e0 + e) + 1] * 4096, 4096 * 8);
#pragma unroll
                for (int u = 0; u < 4; ++u) v[e][u] = ld_sc1(rp, (int64_t)(2 * (tid + POTRF_THREADS * u)) * 8);
            }
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (e < ne) {
                const int q = lists[rec[5] + 3 * (e0 + e)];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int e2 = 2 * (tid + POTRF_THREADS * u), R = 64 * (q >> 1) + (e2 >> 6), C = 64 * (q & 1) + (e2 & 63);
                    if ((R >> 4) >= (C >> 4)) {
                        AT(R, C) += v[e][u].x;
                        AT(R, C + 1) += v[e][u].y;
                    }
                }
            }
    }
    __syncthreads();  // the block final in LDS; the counters and buffers free
    if (tr && threadIdx.x == 0) tr[5] = wall_clock64();
    potrf_body<false, true>(S, ld, j, dinv, scal, nullptr, colflags + j, smem, tr ? tr + 16 : nullptr,
                            rec[9] >= 0 ? P + (int64_t)rec[10] * 4096 : nullptr, rec[9] >= 0 ? fl + rec[9] : nullptr);
#undef AT
}

// split_helper_body (role 4): the tiles of tile columns >= FLOW_CSPLIT of diagonal block j's fused update
// (rec: j, f, -, -, -, -, -, progress flags of the two panel halves of (f, j), flag, scratch slot), from
// the same published rows as the diagonal workgroup, to a scratch partial; then every wave's stores
// drained, a barrier, and one flag (MI355X guide hand-off table row 1)
__device__ __forceinline__ void split_helper_body(double* __restrict__ S, int64_t ld, const int32_t* __restrict__ rec,
                                                  unsigned* __restrict__ fl, double* __restrict__ P,
                                                  double* __restrict__ scal, double* __restrict__ smem,
                                                  uint64_t* __restrict__ tr) {
    const int64_t k0 = (int64_t)rec[1] * CB, f0 = (int64_t)rec[2] * CB;
    const __amdgpu_buffer_rsrc_t rX = block_rsrc(S + k0 * ld + f0, ((int64_t)(CB - 1) * ld + CB) * 8);
    double* Dall = smem + POTRF_NT * IB * 17;
    int* sy = reinterpret_cast<int*>(Dall + (CB / IB) * IB * 17);
    fused_apply<2>(rX, ld, fl + rec[7], rec[8] >= 0 ? fl + rec[8] : nullptr, Dall, reinterpret_cast<double*>(sy + 32), sy, smem,
                   P + (int64_t)rec[10] * 4096, scal, tr);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(fl + rec[9], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tr && threadIdx.x == 0) tr[2] = wall_clock64();
}

// syrk_flow_body (role 2): one update task, C(a, b) quarter q += -sum_k X_ak X_bk' over its sources
// (one elimination-tree level, ascending), each source's column blocks consumed in batches as they are
// published (progress flags of the two panel halves), the whole 128-deep panel in one batch when the
// source is complete.  mode 0: added to C in place after the previous writer of the quarter (rec[9]);
// 1: a split target's partial to scratch, the last group to arrive adds the groups' partials in slot
// order; 2: a late partial to scratch for the diagonal workgroup.  rec[8]: the flag it raises.
__device__ __forceinline__ void syrk_flow_body(double* __restrict__ S, int64_t ld, const int32_t* __restrict__ rec,
                                               const int32_t* __restrict__ lists, double* __restrict__ P,
                                               unsigned* __restrict__ fl, unsigned* __restrict__ cnt,
                                               double* __restrict__ scal, double* __restrict__ smem,
                                               uint64_t* __restrict__ tr) {
    double (*As)[LDW] = reinterpret_cast<double (*)[LDW]>(smem);
    double (*Bs)[LDW] = reinterpret_cast<double (*)[LDW]>(smem + 64 * LDW);
    int* sv = reinterpret_cast<int*>(smem + 128 * LDW);
    const int a = rec[1], b = rec[2], q = rec[3], ns = rec[5], slot = rec[6], mode = rec[7];
    const int32_t* sl = lists + rec[4];
    const int64_t r0 = (int64_t)a * CB + (q >> 1) * 64, c0 = (int64_t)b * CB + (q & 1) * 64;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int lr = lane & 15, lk = lane >> 4;
    const int wr = (wave >> 1) * 16, wc = (wave & 1) * 32;
    const __amdgpu_buffer_rsrc_t rC = block_rsrc(S + r0 * ld + c0, ((int64_t)63 * ld + 64) * 8);
    auto wait_prev = [&]() {
        if (rec[9] >= 0 && tid == 0) spin_ge(fl + rec[9], 1u, scal);
        __syncthreads();
    };
    dbl4 acc[2];
    acc[0] = dbl4{0.0, 0.0, 0.0, 0.0};
    acc[1] = acc[0];
    if (mode == 0) {  // in place: the target (after its previous writer) is the accumulators' start
        wait_prev();
#pragma unroll
        for (int bb = 0; bb < 2; ++bb)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                acc[bb][r] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                                            rC, (int)(((int64_t)(wr + lk + 4 * r) * ld + wc + lr + 16 * bb) * 8), 0, SC1));
    }
    const __amdgpu_buffer_rsrc_t rA = block_rsrc(S + r0 * ld, ((int64_t)63 * ld + ld) * 8);
    const __amdgpu_buffer_rsrc_t rB = block_rsrc(S + c0 * ld, ((int64_t)63 * ld + ld) * 8);
    const int t0 = rec[13], t_end = rec[14];
    // the sources complete at the start (both panel halves have published every column block; thread 0,
    // one flag pair each): such a source's whole panel is prefetched into registers during the previous
    // source's MFMAs, so a many-source task (a dense network's updates) is not load-then-compute per source
    if (tid == 0) {
        unsigned m = 0;
        for (int s = 1; s < ns; ++s)
            if (__hip_atomic_load(fl + sl[3 * s + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)t_end &&
                __hip_atomic_load(fl + sl[3 * s + 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)t_end)
                m |= 1u << s;
        sv[2] = (int)m;
    }
    __syncthreads();
    const unsigned full = (unsigned)sv[2];
    double2 xa[8], xb[8];  // columns [16 t, 16 v) of the 64 rows of A and of B: row item / wpr, column pair item % wpr
    auto load_rng = [&](int s, int t, int v) {
        const int64_t kc = (int64_t)sl[3 * s] * CB;
        const int wpr = 8 * (v - t), nit = 64 * wpr;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = tid + POTRF_THREADS * u;
            if (i < nit) {
                const int row = i / wpr, col = IB * t + 2 * (i % wpr);
                xa[u] = ld_sc1(rA, ((int64_t)row * ld + kc + col) * 8);
                xb[u] = ld_sc1(rB, ((int64_t)row * ld + kc + col) * 8);
            }
        }
    };
    auto store_rng = [&](int t, int v) {
        const int wpr = 8 * (v - t), nit = 64 * wpr;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = tid + POTRF_THREADS * u;
            if (i < nit) {
                const int row = i / wpr, col = IB * t + 2 * (i % wpr);
                As[row][col] = xa[u].x; As[row][col + 1] = xa[u].y;
                Bs[row][col] = xb[u].x; Bs[row][col + 1] = xb[u].y;
            }
        }
    };
    auto compute = [&](int t, int v) {
        for (int kb = IB * t; kb < IB * v; kb += IB) {
            double av[4], b0[4], b1[4];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                av[kk] = -As[wr + lr][kb + 4 * kk + lk];
                b0[kk] = Bs[wc + lr][kb + 4 * kk + lk];
                b1[kk] = Bs[wc + 16 + lr][kb + 4 * kk + lk];
            }
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                acc[0] = mfma(av[kk], b0[kk], acc[0]);
                acc[1] = mfma(av[kk], b1[kk], acc[1]);
            }
        }
    };
    bool held = false;  // xa / xb hold source s's columns [t0, t_end)
    for (int s = 0; s < ns; ++s) {
        if (held) {
            __syncthreads();  // every wave done with the previous source's panel in LDS
            store_rng(t0, t_end);
            __syncthreads();
            held = s + 1 < ns && ((full >> (s + 1)) & 1u);
            if (held) load_rng(s + 1, t0, t_end);
            compute(t0, t_end);
            continue;
        }
        const unsigned* pa = fl + sl[3 * s + 1];
        const unsigned* pb = fl + sl[3 * s + 2];
        int t = t0;
        while (t < t_end) {
            if (tid == 0) {
                unsigned spins = 0, va, vb;
                for (;;) {
                    va = __hip_atomic_load(pa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    vb = __hip_atomic_load(pb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (va > (unsigned)t && vb > (unsigned)t) break;
                    __builtin_amdgcn_s_sleep(1);
                    if (spin_expired(spins, scal)) { va = vb = (unsigned)t_end; break; }
                }
                sv[0] = (int)std::min(std::min(va, vb), (unsigned)t_end);
            }
            __syncthreads();
            const int v = sv[0];
            load_rng(s, t, v);
            store_rng(t, v);
            __syncthreads();
            if (v == t_end && s + 1 < ns && ((full >> (s + 1)) & 1u)) {  // the next source's panel in flight
                load_rng(s + 1, t0, t_end);
                held = true;
            }
            compute(t, v);
            t = v;
        }
    }
    if (tr && tid == 0) tr[4] = wall_clock64();
    auto raise = [&](int32_t flag) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_store(fl + flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    if (mode == 0) {
#pragma unroll
        for (int bb = 0; bb < 2; ++bb)
#pragma unroll
            for (int r = 0; r < 4; ++r) st_sc1(rC, ((int64_t)(wr + lk + 4 * r) * ld + wc + lr + 16 * bb) * 8, acc[bb][r]);
        raise(rec[8]);
        return;
    }
    {   // the partial to its scratch quarter (row-major 64 x 64), write-through
        const __amdgpu_buffer_rsrc_t rP = block_rsrc(P + (int64_t)slot * 4096, 4096 * 8);
#pragma unroll
        for (int bb = 0; bb < 2; ++bb)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                st_sc1(rP, (int64_t)((wr + lk + 4 * r) * 64 + wc + lr + 16 * bb) * 8, acc[bb][r]);
    }
    if (mode == 2) {
        raise(rec[8]);
        return;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
        sv[1] = __hip_atomic_fetch_add(cnt + rec[10], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(rec[12] - 1);
    __syncthreads();
    if (!sv[1]) return;
    wait_prev();  // (its barrier also orders the partial loads below after the arrival)
    double2 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = 2 * (tid + POTRF_THREADS * u), r = e >> 6, cl = e & 63;
        v[u] = ld_sc1(rC, ((int64_t)r * ld + cl) * 8);
    }
    for (int g = 0; g < rec[12]; ++g) {
        const __amdgpu_buffer_rsrc_t rg = block_rsrc(P + (int64_t)(rec[11] + g) * 4096, 4096 * 8);
        double2 pv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) pv[u] = ld_sc1(rg, (int64_t)(2 * (tid + POTRF_THREADS * u)) * 8);
#pragma unroll
        for (int u = 0; u < 4; ++u) { v[u].x += pv[u].x; v[u].y += pv[u].y; }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = 2 * (tid + POTRF_THREADS * u), r = e >> 6, cl = e & 63;
        st_sc1(rC, ((int64_t)r * ld + cl) * 8, v[u]);
    }
    raise(rec[8]);
}

// syrk_block_body (role 2, rec[3] == 4): one update task over a WHOLE off-diagonal target block,
// C(a, b) += -sum_k X_ak X_bk' (128 x 128): per source its 128 rows of A and of B are loaded once for all
// four quarters (half the operand bytes of four quarter tasks), in windows of <= 4 published column blocks
// (LDS: 128 x 64 of each operand).  Eight waves, each 32 rows x 64 columns (2 x 4 tiles of 16 x 16).
// Source entries are 5 ints: k, then the progress flags of A's two panel halves and of B's.  Modes as
// syrk_flow_body: 0 in place after rec[9]; 1 a split target's partial to scratch slots [slot, slot + 4)
// (one 128 x 128 block, row-major), the last group to arrive adds the groups' blocks (slots rec[11] + 4 g)
constexpr int BLK_KW = 64, BLK_LDK = BLK_KW + 2;
constexpr size_t SYRKB_LDS = sizeof(double) * 2 * 128 * BLK_LDK + 16;
__device__ __forceinline__ void syrk_block_body(double* __restrict__ S, int64_t ld, const int32_t* __restrict__ rec,
                                                const int32_t* __restrict__ lists, double* __restrict__ P,
                                                unsigned* __restrict__ fl, unsigned* __restrict__ cnt,
                                                double* __restrict__ scal, double* __restrict__ smem,
                                                uint64_t* __restrict__ tr) {
    double (*As)[BLK_LDK] = reinterpret_cast<double (*)[BLK_LDK]>(smem);
    double (*Bs)[BLK_LDK] = reinterpret_cast<double (*)[BLK_LDK]>(smem + 128 * BLK_LDK);
    int* sv = reinterpret_cast<int*>(smem + 256 * BLK_LDK);
    const int a = rec[1], b = rec[2], ns = rec[5], slot = rec[6], mode = rec[7];
    const int32_t* sl = lists + rec[4];
    const int64_t r0 = (int64_t)a * CB, c0 = (int64_t)b * CB;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int lr = lane & 15, lk = lane >> 4;
    const int wr = (wave >> 1) * 32, wc = (wave & 1) * 64;
    const __amdgpu_buffer_rsrc_t rC = block_rsrc(S + r0 * ld + c0, ((int64_t)127 * ld + 128) * 8);
    dbl4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = dbl4{0.0, 0.0, 0.0, 0.0};
    if (mode == 0) {  // in place: the target (after its previous writer) is the accumulators' start
        if (rec[9] >= 0 && tid == 0) spin_ge(fl + rec[9], 1u, scal);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    acc[i][j][r] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                        rC, (int)(((int64_t)(wr + 16 * i + lk + 4 * r) * ld + wc + 16 * j + lr) * 8), 0, SC1));
    }
    const __amdgpu_buffer_rsrc_t rA = block_rsrc(S + r0 * ld, ((int64_t)127 * ld + ld) * 8);
    const __amdgpu_buffer_rsrc_t rB = block_rsrc(S + c0 * ld, ((int64_t)127 * ld + ld) * 8);
    const int t0 = rec[13], t_end = rec[14];
    // the sources complete at the start (all four panel halves published every column block): their
    // windows need no poll, and the next such window is loaded into registers during this one's MFMAs
    if (tid == 0) {
        unsigned m = 0;
        for (int s = 0; s < ns && s < 32; ++s) {
            bool done = true;
            for (int x = 1; x <= 4; ++x)
                done = done && __hip_atomic_load(fl + sl[5 * s + x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)t_end;
            if (done) m |= 1u << s;
        }
        sv[2] = (int)m;
    }
    __syncthreads();
    const unsigned full = (unsigned)sv[2];
    auto complete = [&](int s) { return s < 32 && ((full >> s) & 1u); };
    double2 xa[8], xb[8];
    auto load_win = [&](int s, int t, int v) {  // rows 0..127 of A and B, columns [16 t, 16 v)
        const int64_t kc = (int64_t)sl[5 * s] * CB;
        const int wpr = 8 * (v - t), nit = 128 * wpr;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = tid + POTRF_THREADS * u;
            if (i < nit) {
                const int row = i / wpr, col = IB * t + 2 * (i % wpr);
                xa[u] = ld_sc1(rA, ((int64_t)row * ld + kc + col) * 8);
                xb[u] = ld_sc1(rB, ((int64_t)row * ld + kc + col) * 8);
            }
        }
    };
    auto store_win = [&](int t, int v) {
        const int wpr = 8 * (v - t), nit = 128 * wpr;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = tid + POTRF_THREADS * u;
            if (i < nit) {
                const int row = i / wpr, col = 2 * (i % wpr);
                As[row][col] = xa[u].x; As[row][col + 1] = xa[u].y;
                Bs[row][col] = xb[u].x; Bs[row][col + 1] = xb[u].y;
            }
        }
    };
    bool held = false;  // xa / xb hold the window (s, t, .) about to be stored
    for (int s = 0; s < ns; ++s) {
        const int32_t* e = sl + 5 * s;
        int t = t0;
        while (t < t_end) {
            int v;
            if (complete(s)) {
                v = std::min(t + BLK_KW / IB, t_end);
            } else {
                if (tid == 0) {  // the column blocks both operands' four panel halves have published
                    unsigned spins = 0, m;
                    for (;;) {
                        m = (unsigned)t_end;
#pragma unroll
                        for (int x = 1; x <= 4; ++x)
                            m = std::min(m, __hip_atomic_load(fl + e[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                        if (m > (unsigned)t) break;
                        __builtin_amdgcn_s_sleep(1);
                        if (spin_expired(spins, scal)) { m = (unsigned)t_end; break; }
                    }
                    sv[0] = (int)m;
                }
                __syncthreads();
                v = std::min(sv[0], t + BLK_KW / IB);  // a window of <= 4 column blocks
            }
            if (!held) load_win(s, t, v);
            store_win(t, v);
            __syncthreads();
            // the next window, when its source is complete: in flight during this window's MFMAs
            held = false;
            if (v < t_end ? complete(s) : (s + 1 < ns && complete(s + 1))) {
                if (v < t_end) load_win(s, v, std::min(v + BLK_KW / IB, t_end));
                else load_win(s + 1, t0, std::min(t0 + BLK_KW / IB, t_end));
                held = true;
            }
            for (int kb = 0; kb < IB * (v - t); kb += IB) {
                double av[2][4], bv[4][4];
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
#pragma unroll
                    for (int i = 0; i < 2; ++i) av[i][kk] = -As[wr + 16 * i + lr][kb + 4 * kk + lk];
#pragma unroll
                    for (int j = 0; j < 4; ++j) bv[j][kk] = Bs[wc + 16 * j + lr][kb + 4 * kk + lk];
                }
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                    for (int i = 0; i < 2; ++i)
#pragma unroll
                        for (int j = 0; j < 4; ++j) acc[i][j] = mfma(av[i][kk], bv[j][kk], acc[i][j]);
            }
            __syncthreads();  // the window is rewritten next
            t = v;
        }
    }
    if (tr && tid == 0) tr[4] = wall_clock64();
    auto raise = [&](int32_t flag) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_store(fl + flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    if (mode == 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    st_sc1(rC, ((int64_t)(wr + 16 * i + lk + 4 * r) * ld + wc + 16 * j + lr) * 8, acc[i][j][r]);
        raise(rec[8]);
        return;
    }
    {   // the partial to its four scratch slots (one row-major 128 x 128 block), write-through
        const __amdgpu_buffer_rsrc_t rP = block_rsrc(P + (int64_t)slot * 4096, 4 * 4096 * 8);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    st_sc1(rP, (int64_t)((wr + 16 * i + lk + 4 * r) * 128 + wc + 16 * j + lr) * 8, acc[i][j][r]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
        sv[1] = __hip_atomic_fetch_add(cnt + rec[10], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(rec[12] - 1);
    __syncthreads();
    if (!sv[1]) return;
    if (rec[9] >= 0 && tid == 0) spin_ge(fl + rec[9], 1u, scal);
    __syncthreads();  // (also orders the partial loads below after the arrival)
    static_assert(POTRF_THREADS * 4 * 2 == 32 * 128, "the combine's 32-row quarters: 4 double2 per thread each");
    for (int h = 0; h < 4; ++h) {  // the block in four 32-row quarters: 4 double2 per thread each
        double2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e2 = 2 * (tid + POTRF_THREADS * u), r = 32 * h + (e2 >> 7), cl = e2 & 127;
            v[u] = ld_sc1(rC, ((int64_t)r * ld + cl) * 8);
        }
        for (int g = 0; g < rec[12]; ++g) {
            const __amdgpu_buffer_rsrc_t rg = block_rsrc(P + (int64_t)(rec[11] + 4 * g) * 4096, 4 * 4096 * 8);
            double2 pv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e2 = 2 * (tid + POTRF_THREADS * u), r = 32 * h + (e2 >> 7), cl = e2 & 127;
                pv[u] = ld_sc1(rg, (int64_t)(r * 128 + cl) * 8);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) { v[u].x += pv[u].x; v[u].y += pv[u].y; }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e2 = 2 * (tid + POTRF_THREADS * u), r = 32 * h + (e2 >> 7), cl = e2 & 127;
            st_sc1(rC, ((int64_t)r * ld + cl) * 8, v[u]);
        }
    }
    raise(rec[8]);
}

constexpr size_t FLOW_LDS_A = FLOWF_LDS > TRSMF_LDS ? FLOWF_LDS : TRSMF_LDS;
constexpr size_t FLOW_LDS_B0 = SYRKW_LDS > TRTRI_LDS ? SYRKW_LDS : TRTRI_LDS;
constexpr size_t FLOW_LDS_B = FLOW_LDS_B0 > SYRKB_LDS ? FLOW_LDS_B0 : SYRKB_LDS;
constexpr size_t FLOW_LDS = FLOW_LDS_A > FLOW_LDS_B ? FLOW_LDS_A : FLOW_LDS_B;
static_assert(FLOW_LDS + 16 <= 160 * 1024, "k_chol_flow LDS (+ the static ticket word)");
static_assert(SYRKW_LDS >= sizeof(double) * 128 * LDW + 3 * sizeof(int), "syrk_flow_body broadcast words");

__device__ __forceinline__ void flow_record(int rid, double* __restrict__ S, int64_t ld, const int32_t* __restrict__ lists,
                                            const int32_t* __restrict__ recs, double* __restrict__ dinv,
                                            double* __restrict__ linv, double* __restrict__ scal,
                                            unsigned* __restrict__ colflags, unsigned* __restrict__ fl,
                                            unsigned* __restrict__ cnt, double* __restrict__ P,
                                            uint64_t* __restrict__ trace, double* __restrict__ gblk,
                                            double* __restrict__ smem) {
    const int32_t* rec = recs + Sched::FLOW_REC * (int64_t)rid;
    uint64_t* tr = trace ? trace + FTRACE * (int64_t)rid : nullptr;
    if (tr && threadIdx.x == 0) tr[0] = wall_clock64();
    const int role = rec[0];
    if (role == 0) {
        diag_body(S, ld, rec, lists, dinv, scal, colflags, fl, P, smem, tr);
    } else if (role == 1) {
        wait_list_sc1(lists + rec[3], rec[4], fl, scal);  // the final writers of the panel block's quarters
        if (tr && threadIdx.x == 0) tr[1] = wall_clock64();
        trsm_flow_body(S, ld, rec + 1, dinv, colflags + rec[1], scal, smem, tr, fl + rec[5],
                       (gblk && rec[7] >= 0) ? gblk + (int64_t)rec[7] * 256 : nullptr);
    } else if (role == 2) {
        if (rec[3] == 4) syrk_block_body(S, ld, rec, lists, P, fl, cnt, scal, smem, tr);
        else syrk_flow_body(S, ld, rec, lists, P, fl, cnt, scal, smem, tr);
    } else if (role == 4) {
        split_helper_body(S, ld, rec, fl, P, scal, smem, tr);
    } else {
        if (threadIdx.x == 0) spin_ge(colflags + rec[1], (unsigned)(CB / IB), scal);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        trtri_body(S, ld, rec[1], dinv, linv, smem);
    }
    if (tr) {
        __syncthreads();
        if (threadIdx.x == 0) {
            tr[2] = wall_clock64();
            tr[3] = (uint64_t)role | ((uint64_t)(uint32_t)rec[1] << 8) | ((uint64_t)(uint32_t)rec[2] << 32);
        }
    }
}

__global__ __launch_bounds__(POTRF_THREADS) void k_chol_flow(double* __restrict__ S, int64_t ld,
                                                             const int32_t* __restrict__ lists,
                                                             const int32_t* __restrict__ recs,
                                                             double* __restrict__ dinv, double* __restrict__ linv,
                                                             double* __restrict__ scal, unsigned* __restrict__ colflags,
                                                             unsigned* __restrict__ fl, unsigned* __restrict__ cnt,
                                                             double* __restrict__ P, uint64_t* __restrict__ trace,
                                                             double* __restrict__ gblk, unsigned* __restrict__ ticket) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    __shared__ int s_ticket;
    const uint64_t t_wg = trace ? wall_clock64() : 0;
    if (threadIdx.x == 0) {
        // static order: the record comes from an atomic ticket, not from blockIdx: tickets follow the
        // order in which the workgroups really start, and every record waits only for records of smaller
        // index (build_flow's order check), so each wait points to a workgroup that has already started
        // and is resident (or done) -- progress does not depend on the hardware dispatching blockIdx in
        // order, nor on every record being co-resident.  (Measured and not kept, round 5: the critical
        // records -- diagonal blocks, panel halves, split helpers -- and the others in two queues, each a
        // subsequence of this order, (a) on a persistent grid of one workgroup per CU, K of them for the
        // critical queue: 1,122-1,297 us per launch at config 4 for K = 48..176 vs 451 us, the record
        // bodies inside the workgroup's loop spilling 2,320 B per lane; (b) one workgroup per record with
        // a budget of K resident critical records and #CU - K others: 580-868 us for K = 32..128, and a
        // hand-off timeout at K = 176 -- the update queue runs ahead of the critical one, whose budget
        // then throttles the wide lower levels.)
        s_ticket = (int)__hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // a record that starts after a hand-off timeout is skipped (its inputs may never be published)
    if (threadIdx.x == 0 && s_ticket >= 0 && hand_off_aborted(scal)) s_ticket = -1;
    __syncthreads();
    const int rid = s_ticket;
    if (rid < 0) return;
    if (trace && threadIdx.x == 0) trace[FTRACE * (int64_t)rid + 48] = t_wg;
    flow_record(rid, S, ld, lists, recs, dinv, linv, scal, colflags, fl, cnt, P, trace, gblk, smem);
}

// ------------------------------------------------------------------------------------------------
// backward solve L' x = y with the diagonal-block inverses:
//   k_bwd_first  x_{nb-1} = Linv_{nb-1}^T y_{nb-1}
//   k_bwd_step   (kb): workgroup 0 (the critical one) y_{kb-1} -= L_{kb,kb-1}^T x_kb and then
//                x_{kb-1} = Linv_{kb-1}^T y_{kb-1}; workgroup 1+j updates y_j -= L_{kb,j}^T x_kb
// 256 threads = 128 columns x 2 halves of the 128 rows, halves summed in a fixed order.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ double gemv_t128(const double* __restrict__ M, int64_t ldm, const double* __restrict__ v,
                                            int tid, double* red) {
    // thread -> columns 2 (tid & 63) + {0,1}, rows 32 (tid >> 6) .. +32: all 32 double2 loads in flight
    const int c2 = tid & 63, h = tid >> 6;
    double2 m[32];
#pragma unroll
    for (int r = 0; r < 32; ++r) m[r] = *reinterpret_cast<const double2*>(M + (int64_t)(h * 32 + r) * ldm + 2 * c2);
    double a0 = 0.0, a1 = 0.0;
#pragma unroll
    for (int r = 0; r < 32; ++r) {
        const double vr = v[h * 32 + r];
        a0 += m[r].x * vr;
        a1 += m[r].y * vr;
    }
    red[h * 128 + 2 * c2] = a0;
    red[h * 128 + 2 * c2 + 1] = a1;
    __syncthreads();
    const int c = tid & 127;
    const double s = (red[c] + red[128 + c]) + (red[256 + c] + red[384 + c]);
    __syncthreads();
    return s;  // valid for every thread (column c = tid & 127)
}

// k_bwd_wave: one level of the backward solve (levels run top down).  Workgroup b < nsrc: column
// i = srcs[b] of the level, x_i = Linv_i' y_i (y_i is final: its contributions came from higher
// levels).  Workgroup nsrc + t: target column j = tgts[t], y_j -= sum_i L(i,j)' x_i over its sources
// (ascending; x_i recomputed locally from y_i, one 128x128 GEMV, instead of a second launch).
// (blockIdx.y = r: right-hand-side row yrow + r, solution X + r xstride -- several rows per launch)
__global__ __launch_bounds__(256) void k_bwd_wave(double* __restrict__ S, int64_t ld, int64_t yrow,
                                                  const double* __restrict__ linv, double* __restrict__ X,
                                                  const int32_t* __restrict__ srcs, int nsrc,
                                                  const int32_t* __restrict__ tgts, const int32_t* __restrict__ tstart,
                                                  const int32_t* __restrict__ tsrc, int64_t xstride = 0) {
    __shared__ double ys[CB];
    __shared__ double xs[CB];
    __shared__ double red[512];
    const int tid = threadIdx.x;
    X += (int64_t)blockIdx.y * xstride;
    double* y = S + (yrow + blockIdx.y) * ld;  // the right-hand-side row (n_pad: the solve; n_pad + a: border column a)
    if ((int)blockIdx.x < nsrc) {
        const int64_t i = srcs[blockIdx.x];
        if (tid < CB) ys[tid] = y[i * CB + tid];
        __syncthreads();
        const double x = gemv_t128(linv + i * CB * CB, CB, ys, tid, red);
        if (tid < CB) X[i * CB + tid] = x;
        return;
    }
    const int t = blockIdx.x - nsrc;
    const int64_t j = tgts[t];
    double acc = 0.0;
    for (int q = tstart[t]; q < tstart[t + 1]; ++q) {
        const int64_t i = tsrc[q];
        if (tid < CB) ys[tid] = y[i * CB + tid];
        __syncthreads();
        const double x = gemv_t128(linv + i * CB * CB, CB, ys, tid, red);
        if (tid < CB) xs[tid] = x;
        __syncthreads();
        acc += gemv_t128(S + i * CB * ld + j * CB, ld, xs, tid, red);
    }
    if (tid < CB) y[j * CB + tid] -= acc;
}

// k_bwd_flow: the whole backward solve L' x = y in ONE launch, dataflow-ordered: workgroup b owns
// block column j = nb-1-b; it stages Linv_j in LDS, then for each source block row i of column j
// (descending: the order the x_i are published in) streams L(i,j) into registers, polls x_i itself
// (sc1 loads until no value is X_SENTINEL, which k_border_rhs wrote) and adds L(i,j)' x_i; then
// x_j = Linv_j' (y_j - sum), published write-through, and delta_c = -x_j stored (k_neg_copy fused).  Roles
// come from an atomic ticket in start order and waits only point to higher blocks (earlier tickets), so
// they end whether or not the whole grid is co-resident; polls are
// bounded (scal[1] = -1 on timeout, reported by the host).
// With inner constraints and `combine`, one more workgroup (ticket 0) solves the border's 14x14
// system (border_combine_body) meanwhile, publishes the coefficients write-through and raises flags[nb];
// the block workgroups wait for it only where they form u_j (after staging and their sources).
constexpr size_t BWD_LDS = sizeof(double) * (CB * CB + (CB / IB) * IB * IB + 2 * CB + 512 + 16);
static_assert(BWD_LDS + 16 <= 160 * 1024, "k_bwd_flow LDS (+ the static ticket word)");

__global__ __launch_bounds__(256) void k_bwd_flow(const double* __restrict__ S, int64_t ld, int64_t n_pad,
                                                  const double* __restrict__ linv, const double* __restrict__ dinv,
                                                  double* __restrict__ X,
                                                  double* __restrict__ delta, int64_t u_c,
                                                  const int32_t* __restrict__ src_start, const int32_t* __restrict__ src,
                                                  unsigned* __restrict__ flags, double* __restrict__ scal,
                                                  double* __restrict__ coef, int combine,
                                                  const double* __restrict__ gpart, const double* __restrict__ gblk, int nblk,
                                                  unsigned* __restrict__ ticket, const int8_t* __restrict__ bown,
                                                  const double* __restrict__ bsc) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* Li = smem;              // [128][128] Linv_j, or L_jj for a root column
    double* Dt = Li + CB * CB;      // [8][16][16] the leaf inverses of a root column (else: partial sums)
    double* xs = Dt + (CB / IB) * IB * IB;  // [128] x_i of the current source
    double* ys = xs + CB;           // [128]
    double* red = ys + CB;          // [512]
    double* cs = red + 512;         // [16] the border coefficients
    const int tid = threadIdx.x;
    const int nb = (int)(n_pad / CB);
    // roles by atomic ticket (real start order): ticket 0 is the border combine (when present), then
    // the block columns top down -- every wait (a higher block's x, the combine's coefficients) points
    // to a workgroup that started earlier, so progress needs neither in-order dispatch nor co-residency
    __shared__ int s_ticket;
    if (tid == 0) {
        s_ticket = (int)__hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (hand_off_aborted(scal)) s_ticket = -1;  // the factorisation timed out: nothing to solve
    }
    __syncthreads();
    const int tk = s_ticket;
    if (tk < 0) return;
    if (combine && tk == 0) {  // the border combine workgroup
        border_combine_body(gpart, gblk, nblk, reinterpret_cast<double (*)[15]>(Li), cs, bsc);
        if (tid < 14) {
            const __amdgpu_buffer_rsrc_t rc = block_rsrc(coef, 16 * 8);
            st_sc1(rc, (int64_t)tid * 8, cs[tid]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_store(flags + nb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    const int j = nb - 1 - (tk - combine);
    // (subtree split: another rank's subtree column -- nothing of this rank depends on it)
    if (bown && bown[j] == 0) return;
    const int c2 = tid & 63, h = tid >> 6;  // gemv_t128's thread map: columns 2 c2 + {0,1}, rows 32 h ..
    // a root of the elimination tree (no source blocks: the top level) is solved by substitution with
    // its factor and leaf inverses, so its Linv (k_trtri128, 30 us) is off the critical path
    const bool root = src_start[j] == src_start[j + 1];
    {
        const double2* Lg = root ? nullptr : reinterpret_cast<const double2*>(linv + (int64_t)j * CB * CB);
        double2* Ls = reinterpret_cast<double2*>(Li);
        for (int q = tid; q < CB * CB / 2; q += 256) {
            const int r = q >> 6, cc = (q & 63) * 2;
            Ls[q] = root ? *reinterpret_cast<const double2*>(S + ((int64_t)j * CB + r) * ld + (int64_t)j * CB + cc) : Lg[q];
        }
        if (root)
            for (int q = tid; q < (CB / IB) * IB * IB; q += 256) Dt[q] = dinv[(int64_t)j * (CB / IB) * IB * IB + q];
    }
    // u_j = y_j + F_j c (the inner-constraint combine, coefficients cs) does not depend on the sources:
    // formed ahead of them, off the chain of published x blocks (the coefficients come from the combine
    // workgroup, an earlier ticket, or a previous launch)
    // (row ur of thread tid: tid for a root, whose substitution reads y from LDS; else row 32 h + (lane & 31),
    // so that wave h forms the 32 entries of y_j its rows of the final product need without another barrier)
    const int ur = root ? tid : 32 * h + (c2 & 31);
    const bool uown = ur < CB;
    double u = 0.0;
    if (uown) u = S[n_pad * ld + (int64_t)j * CB + ur];
    if (coef) {
        double f[14];
        if (uown)
#pragma unroll
            for (int m = 0; m < 14; ++m) f[m] = S[(n_pad + 1 + m) * ld + (int64_t)j * CB + ur];
        if (combine && tid == 0) {
            unsigned spins = 0;
            while (__hip_atomic_load(flags + nb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 1u) {
                __builtin_amdgcn_s_sleep(1);
                if (spin_expired(spins, scal)) break;
            }
        }
        __syncthreads();
        if (tid < 7) {
            const double2 v = ld_sc1(block_rsrc(coef, 16 * 8), (int64_t)(2 * tid) * 8);
            cs[2 * tid] = v.x;
            cs[2 * tid + 1] = v.y;
        }
        __syncthreads();
        if (uown)
#pragma unroll
            for (int m = 0; m < 14; ++m) u += f[m] * cs[m];
    }
    double a0 = 0.0, a1 = 0.0;
    const __amdgpu_buffer_rsrc_t rX = block_rsrc(X, n_pad * 8);
    for (int q = src_start[j]; q < src_start[j + 1]; ++q) {
        const int i = src[q];
        const double* M = S + (int64_t)i * CB * ld + (int64_t)j * CB;  // L(i, j), written by earlier launches
        double2 m[32];
#pragma unroll
        for (int r = 0; r < 32; ++r) m[r] = *reinterpret_cast<const double2*>(M + (int64_t)(h * 32 + r) * ld + 2 * c2);
        // each wave polls the 32 values of x_i its rows need (sc1; lane l holds 2 (l & 15), + 1) until none
        // is the sentinel, and takes them lane by lane (readlane): no workgroup barrier per source
        unsigned spins = 0;
        double2 v;
        for (;;) {
            asm volatile("" ::: "memory");  // the load is re-issued every spin (not hoisted)
            v = ld_sc1(rX, ((int64_t)i * CB + h * 32 + 2 * (c2 & 15)) * 8);
            const bool ok = __builtin_bit_cast(uint64_t, v.x) != X_SENTINEL && __builtin_bit_cast(uint64_t, v.y) != X_SENTINEL;
            if (__all(ok)) break;
            __builtin_amdgcn_s_sleep(1);
            if (spin_expired(spins, scal)) break;
        }
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            const double xr = readlane_d((r & 1) ? v.y : v.x, r >> 1);
            a0 += m[r].x * xr;
            a1 += m[r].y * xr;
        }
    }
    red[h * 128 + 2 * c2] = a0;
    red[h * 128 + 2 * c2 + 1] = a1;
    __syncthreads();
    const double yu = uown ? u - ((red[ur] + red[128 + ur]) + (red[256 + ur] + red[384 + ur])) : 0.0;
    if (root) {
        if (tid < CB) ys[tid] = yu;
        __syncthreads();
        // x = L^-T y by substitution in wave 0 alone (no workgroup barriers): tiles s = 7 .. 0,
        // x_s = D_s' (y_s - sum_{t>s} L_ts' x_t); lane (c = lane & 15, quarter g = lane >> 4) sums the
        // rows g, g+4, .. below tile s for column c, the quarters added by a fixed xor butterfly
        if (tid < 64) {
            const int c = tid & 15, g = tid >> 4;
            for (int sb = CB / IB - 1; sb >= 0; --sb) {
                double a = 0.0;
                for (int r = IB * (sb + 1) + g; r < CB; r += 4) a += Li[r * CB + IB * sb + c] * xs[r];
                a += __shfl_xor(a, 16, 64);
                a += __shfl_xor(a, 32, 64);
                const double rs = ys[IB * sb + c] - a;  // every quarter holds r_s[c]
                double x = 0.0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {             // (D_s' r)[c] = sum_r D_s[r][c] r[r], r = 4 g + q
                    const int r = 4 * g + q;
                    x += Dt[sb * IB * IB + r * IB + c] * __shfl(rs, r, 64);
                }
                x += __shfl_xor(x, 16, 64);
                x += __shfl_xor(x, 32, 64);
                if (g == 0) xs[IB * sb + c] = x;
                __builtin_amdgcn_s_waitcnt(0xC07F);
                __builtin_amdgcn_wave_barrier();
            }
        }
        __syncthreads();
        if (tid < CB) {
            const double x = xs[tid];
            st_sc1(rX, ((int64_t)j * CB + tid) * 8, x);
            const int64_t g = (int64_t)j * CB + tid;
            if (g < u_c) delta[g] = -x;
        }
        return;
    }
    // x_j = Linv_j' y_j from LDS, y_j's row 32 h + r from lane r of wave h; the partial sums go to the
    // leaf-inverse area (a root's only), as other waves may still read `red`
    double b0 = 0.0, b1 = 0.0;
#pragma unroll 8
    for (int r = 0; r < 32; ++r) {
        const double yr = readlane_d(yu, r);
        const double2 l = *reinterpret_cast<const double2*>(Li + (h * 32 + r) * CB + 2 * c2);
        b0 += l.x * yr;
        b1 += l.y * yr;
    }
    double* red2 = Dt;
    red2[h * 128 + 2 * c2] = b0;
    red2[h * 128 + 2 * c2 + 1] = b1;
    __syncthreads();
    if (tid < CB) {
        const double x = (red2[tid] + red2[128 + tid]) + (red2[256 + tid] + red2[384 + tid]);
        st_sc1(rX, ((int64_t)j * CB + tid) * 8, x);
        const int64_t g = (int64_t)j * CB + tid;
        if (g < u_c) delta[g] = -x;
    }
}

__global__ void k_neg_copy(const double* __restrict__ X, double* __restrict__ delta, int64_t u_c) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < u_c) delta[i] = -X[i];
}

// ------------------------------------------------------------------------------------------------
// One batched step per elimination-tree level (fba_order.cpp): potrf of the level's diagonal blocks,
// the panel solves of their columns (RHS block row included: the forward solve), the trailing
// updates they cause.  Three launches per level on one stream.
// ------------------------------------------------------------------------------------------------
// part (subtree split): 0 = this rank's subtree columns (flow A), 1 = the top columns (flow B, its
// flag / counter / scratch ids after flow A's, its own start ticket)
int launch_cholesky(Ctx& c, int part) {
    const int64_t ld = c.L.ld;
    const Sched& s = c.sched;
    if (s.split) {
        const Sched::FlowPart& T = s.top;
        const bool b = part == 1;
        const int n = b ? T.n : s.flow_n;
        if (n == 0) return FBA_OK;
        const int64_t fo = b ? s.flow_nprog + s.flow_nuflag : 0, co = b ? s.flow_ncounter : 0, so = b ? s.flow_nscratch : 0;
        const bool pp = c.probe == 2 && c.probe_n < (int)c.probe_ev.size() / 2;
        if (pp) FBA_HIP(hipEventRecord(c.probe_ev[2 * c.probe_n], c.stream));
        k_chol_flow<<<(unsigned)n, POTRF_THREADS, FLOW_LDS, c.stream>>>(
            c.d_S, ld, c.d_sched, c.d_sched + (b ? T.rec : s.flow_rec), c.d_dinv, c.d_linv, c.d_scal, c.d_flags,
            c.d_tflags + fo, c.d_counters + co, c.d_P + so * 4096, nullptr, c.set.inner_constraints ? c.d_gblk : nullptr,
            c.d_tickets + (b ? 2 : 0));
        if (pp) {
            FBA_HIP(hipEventRecord(c.probe_ev[2 * c.probe_n + 1], c.stream));
            c.probe_flops += b ? T.flops : s.flow_flops;
            ++c.probe_n;
        }
        FBA_HIP(hipGetLastError());
        return FBA_OK;
    }
    if (c.chol_flow && s.flow_ok && s.flow_n > 0) {
        // the whole factorisation + forward solve in one persistent launch (flags zeroed by k_border_rhs)
        const bool pp = c.probe == 2 && c.probe_n < (int)c.probe_ev.size() / 2;
        if (pp) FBA_HIP(hipEventRecord(c.probe_ev[2 * c.probe_n], c.stream));
        k_chol_flow<<<(unsigned)s.flow_n, POTRF_THREADS, FLOW_LDS, c.stream>>>(
            c.d_S, ld, c.d_sched, c.d_sched + s.flow_rec, c.d_dinv, c.d_linv, c.d_scal, c.d_flags, c.d_tflags,
            c.d_counters, c.d_P, c.d_ptrace, c.set.inner_constraints ? c.d_gblk : nullptr, c.d_tickets);
        if (pp) {
            FBA_HIP(hipEventRecord(c.probe_ev[2 * c.probe_n + 1], c.stream));
            c.probe_flops += s.flow_flops;
            ++c.probe_n;
        }
        FBA_HIP(hipGetLastError());
        return FBA_OK;
    }
    // the k_panel / k_bwd_flow hand-off flags, the split-target counters and the update flags were
    // zeroed by k_border_rhs
    int pend = -1;  // a level whose trailing updates run inside the next level's k_panel
    auto updates = [&](int v) -> int {  // a level's trailing updates as their own launch
        const Sched::Wave& V = s.w[v];
        const bool pr = c.probe == 1 && c.probe_n < (int)c.probe_ev.size() / 2;
        if (pr) FBA_HIP(hipEventRecord(c.probe_ev[2 * c.probe_n], c.stream));
        k_syrk_multi<<<(unsigned)V.ntask, 256, 0, c.stream>>>(c.d_S, ld, c.d_sched + V.tasks, c.d_sched + V.src, c.d_P,
                                                               c.d_sched + V.comb, c.d_counters + V.cbase);
        if (pr) {
            FBA_HIP(hipEventRecord(c.probe_ev[2 * c.probe_n + 1], c.stream));
            c.probe_flops += V.flops;
            ++c.probe_n;
        }
        return FBA_OK;
    };
    for (int w = 0; w < s.n_waves; ++w) {
        const Sched::Wave& W = s.w[w];
        const int nprev = w > 0 ? s.w[w - 1].ncol : 0;  // the previous level's blocks, inverted alongside
        const int32_t* prev = c.d_sched + (w > 0 ? s.w[w - 1].cols : 0);
        const bool fits = W.ncol + W.ntrsm + nprev <= c.n_cu;  // potrf + panel solves resident (one per CU)
        if (pend >= 0 && !fits) { updates(pend); pend = -1; }
        const Sched::Wave* U = pend >= 0 ? &s.w[pend] : nullptr;
        const bool pp = c.probe == 2 && c.probe_n < (int)c.probe_ev.size() / 2;
        if (pp) FBA_HIP(hipEventRecord(c.probe_ev[2 * c.probe_n], c.stream));
        if (fits) {
            // one launch: [U's updates of this level's diagonal blocks][potrf][U's other updates]
            // [panel solves][inverses of the previous level's blocks]; U = the previous level (merged)
            k_panel<<<(unsigned)(W.ncol + W.ntrsm + nprev + (U ? U->ntask : 0)), POTRF_THREADS, PANEL_LDS, c.stream>>>(
                c.d_S, ld, c.d_sched + W.cols, W.ncol, c.d_sched + W.trsm, W.ntrsm, prev, nprev, c.d_dinv, c.d_linv,
                c.d_scal, c.d_flags, (int)c.panel_progressive, U ? c.d_sched + U->tasks : nullptr, U ? U->ntask : 0,
                U ? U->ndiag : 0, U ? U->npanel : 0, U ? c.d_sched + U->src : nullptr, c.d_P,
                U ? c.d_sched + U->comb : nullptr,
                U ? c.d_counters + U->cbase : nullptr, c.d_tflags, c.d_sched + W.wstart, c.d_sched + W.wlist,
                c.d_ptrace ? c.d_ptrace + (int64_t)w * PTRACE_WG * 8 : nullptr);
        } else {
            k_potrf128<false><<<(unsigned)W.ncol, POTRF_THREADS, POTRF_LDS, c.stream>>>(c.d_S, ld, c.d_sched + W.cols,
                                                                                      c.d_dinv, c.d_scal, nullptr);
            k_trsm128<<<(unsigned)W.ntrsm, 256, TRSM_LDS, c.stream>>>(c.d_S, ld, c.d_sched + W.trsm, c.d_dinv);
            if (nprev > 0)
                k_trtri128<<<(unsigned)nprev, 256, TRTRI_LDS, c.stream>>>(c.d_S, ld, prev, c.d_dinv, c.d_linv);
        }
        if (pp) {
            FBA_HIP(hipEventRecord(c.probe_ev[2 * c.probe_n + 1], c.stream));
            c.probe_flops += W.pflops + (U ? U->flops : 0.0);
            ++c.probe_n;
        }
        pend = -1;
        if (W.ntask == 0) continue;
        if (c.merge_updates) pend = w;  // into the next level's k_panel
        else updates(w);
    }
    if (pend >= 0) updates(pend);
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

// backward solves of the forward-solved right-hand-side rows row0 .. row0+nrows-1 (covariance,
// fba_cov.hip); X + r n_pad receives the solution of row row0 + r.  The rows are consumed.
int launch_backward_rows(Ctx& c, int row0, int nrows, double* X) {
    const int64_t ld = c.L.ld;
    const Sched& s = c.sched;
    for (int w = s.n_waves - 1; w >= 0; --w) {  // all rows of a level in one launch
        const Sched::BWave& B = s.b[w];
        k_bwd_wave<<<dim3((unsigned)(B.nsrc + B.ntgt), (unsigned)nrows), 256, 0, c.stream>>>(
            c.d_S, ld, c.L.n_pad + row0, c.d_linv, X, c.d_sched + B.srcs, B.nsrc, c.d_sched + B.tgts,
            c.d_sched + B.src_start, c.d_sched + B.src, c.L.n_pad);
    }
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

// test hook (fba_test_border_solve): k_border_combine's 14x14 solve for a given 15x15 Gram matrix,
// placed in Gram segment 0 (the other segments zero)
int border_solve_selftest(int device, const double* gram, double* coef) {
    FBA_HIP(hipSetDevice(device));
    std::vector<double> gp((size_t)GRAM_SEG * 120, 0.0);
    for (int e = 0, a = 0; a < 15; ++a)
        for (int b = a; b < 15; ++b, ++e) gp[e] = gram[a * 15 + b];
    double *dg = nullptr, *dc = nullptr;
    FBA_HIP(hipMalloc((void**)&dg, gp.size() * sizeof(double)));
    hipError_t e1 = hipMalloc((void**)&dc, 16 * sizeof(double));
    if (e1 == hipSuccess) e1 = hipMemcpy(dg, gp.data(), gp.size() * sizeof(double), hipMemcpyHostToDevice);
    if (e1 == hipSuccess) {
        k_border_combine<<<1, 256>>>(nullptr, 0, 0, dg, dc);
        e1 = hipGetLastError();
    }
    if (e1 == hipSuccess) e1 = hipMemcpy(coef, dc, 14 * sizeof(double), hipMemcpyDeviceToHost);
    (void)hipFree(dg);
    if (dc) (void)hipFree(dc);
    FBA_HIP(e1);
    return FBA_OK;
}

int launch_border_gram(Ctx& c, double* gpart, int* nseg) {
    k_border_gram<<<GRAM_SEG, 256, 0, c.stream>>>(c.d_S, c.L.ld, c.L.n_pad, gpart);
    *nseg = GRAM_SEG;
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

// the diagonal-block inverses of the last level (the others come from the next level's k_panel)
int launch_trtri_last(Ctx& c) {
    const Sched& s = c.sched;
    if (s.n_waves > 0)
        k_trtri128<<<(unsigned)s.w[s.n_waves - 1].ncol, 256, TRTRI_LDS, c.stream>>>(
            c.d_S, c.L.ld, c.d_sched + s.w[s.n_waves - 1].cols, c.d_dinv, c.d_linv);
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int launch_backward(Ctx& c) {
    int rc;
    const int64_t ld = c.L.ld;
    const Sched& s = c.sched;
    const int64_t nb = c.L.n_pad / CB;
    const bool flow = c.bwd_flow;  // (ticket-ordered roles: no co-residency requirement)
    double* coef = c.d_bscr + 32 * 14 + 16 * 120;
    const bool gblk = c.chol_flow && s.flow_ok && (s.flow_n > 0 || s.split);
    // the combine inside k_bwd_flow (one more workgroup) when the Gram comes from k_chol_flow
    const int combine = (c.set.inner_constraints && flow && gblk) ? 1 : 0;
    if (c.set.inner_constraints && !combine) {
        // (running k_trtri128 on a forked stream concurrently with these two measured slower: a forked
        // iteration graph adds cross-queue waits to every launch of the Cholesky chain)
        // k_chol_flow's RHS panel halves left the Gram as per-block partials (d_gblk); otherwise
        // k_border_gram forms it from the forward-solved rows
        if (!gblk) k_border_gram<<<GRAM_SEG, 256, 0, c.stream>>>(c.d_S, ld, c.L.n_pad, c.d_bscr + 32 * 14);
        if (flow)  // the 14 coefficients only; k_bwd_flow applies them to its block
            k_border_combine<<<1, 256, 0, c.stream>>>(c.d_S, ld, c.L.n_pad, c.d_bscr + 32 * 14, coef,
                                                      gblk ? c.d_gblk : nullptr, (int)nb);
        else
            k_border_combine<<<(unsigned)((c.L.n_pad + 255) / 256), 256, 0, c.stream>>>(c.d_S, ld, c.L.n_pad,
                                                                                       c.d_bscr + 32 * 14, nullptr, gblk ? c.d_gblk : nullptr, (int)nb);
    }
    if (flow) {  // one launch, every workgroup resident; roots solve by substitution
        k_bwd_flow<<<(unsigned)(nb + combine), 256, BWD_LDS, c.stream>>>(
            c.d_S, ld, c.L.n_pad, c.d_linv, c.d_dinv, c.d_X, c.d_delta, c.L.u_c, c.d_sched + s.bf_start,
            c.d_sched + s.bf_src, c.d_bflags, c.d_scal, c.set.inner_constraints ? coef : nullptr, combine,
            c.d_bscr + 32 * 14, c.d_gblk, (int)nb, c.d_tickets + 1, s.split ? c.d_bown : nullptr,
            s.split ? c.d_bscr + BSC_OFF : nullptr);
        FBA_HIP(hipGetLastError());
        return FBA_OK;
    }
    if ((rc = launch_trtri_last(c))) return rc;
    for (int w = s.n_waves - 1; w >= 0; --w) {
        const Sched::BWave& B = s.b[w];
        k_bwd_wave<<<(unsigned)(B.nsrc + B.ntgt), 256, 0, c.stream>>>(c.d_S, ld, c.L.n_pad, c.d_linv, c.d_X,
                                                                     c.d_sched + B.srcs, B.nsrc, c.d_sched + B.tgts,
                                                                     c.d_sched + B.src_start, c.d_sched + B.src);
    }
    k_neg_copy<<<(unsigned)((c.L.u_c + 255) / 256), 256, 0, c.stream>>>(c.d_X, c.d_delta, c.L.u_c);
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int chol_setup(Ctx& c) {
    FBA_HIP(hipFuncSetAttribute((const void*)k_potrf128<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)POTRF_LDS));
    FBA_HIP(hipFuncSetAttribute((const void*)k_trsm128, hipFuncAttributeMaxDynamicSharedMemorySize, (int)TRSM_LDS));
    FBA_HIP(hipFuncSetAttribute((const void*)k_panel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)PANEL_LDS));
    FBA_HIP(hipFuncSetAttribute((const void*)k_chol_flow, hipFuncAttributeMaxDynamicSharedMemorySize, (int)FLOW_LDS));
    // FBA_CHOL_FLOW=0: the level-by-level k_panel launches instead of the persistent dataflow launch
    c.chol_flow = !(getenv("FBA_CHOL_FLOW") && atoi(getenv("FBA_CHOL_FLOW")) == 0);
    static_assert(TRSM_LDS >= POTRF_LDS, "k_panel LDS");
    hipDeviceProp_t prop;
    FBA_HIP(hipGetDeviceProperties(&prop, c.device));
    c.n_cu = prop.multiProcessorCount;
    // (one more than the blocks: k_bwd_flow's border-combine flag; a multiple of 16 bytes)
    c.flags_bytes = (size_t)((c.L.n_pad / CB + 1 + 3) / 4 * 4) * sizeof(unsigned);
    const size_t nf = c.flags_bytes / sizeof(unsigned);
    // [flags][bflags][split-target counters][update flags][3 tickets: k_chol_flow, k_bwd_flow, flow B]
    c.n_sync = (int64_t)(2 * nf + std::max(c.sched.n_counters, 1) + std::max(c.sched.n_tflags, 1) + 3);
    FBA_HIP(hipMalloc((void**)&c.d_flags, sizeof(unsigned) * c.n_sync));
    FBA_HIP(hipMemset(c.d_flags, 0, sizeof(unsigned) * c.n_sync));
    c.d_bflags = c.d_flags + nf;
    c.d_counters = c.d_bflags + nf;
    c.d_tflags = c.d_counters + std::max(c.sched.n_counters, 1);
    c.d_tickets = c.d_tflags + std::max(c.sched.n_tflags, 1);
    // FBA_BWD_LEVELS=1: the level-by-level backward solve (k_bwd_wave) instead of k_bwd_flow
    c.bwd_flow = !(getenv("FBA_BWD_LEVELS") && atoi(getenv("FBA_BWD_LEVELS")) != 0);
    // the subtree split runs flow A / flow B of k_chol_flow and k_bwd_flow's ownership masks and border
    // scales: the per-level paths (k_panel, k_bwd_wave + k_border_combine + k_neg_copy) know neither
    if (c.sched.split && (!c.chol_flow || !c.bwd_flow || !c.sched.flow_ok || !c.sched.top.ok)) {
        set_error("subtree split needs the k_chol_flow / k_bwd_flow schedules (FBA_CHOL_FLOW and FBA_BWD_LEVELS unset)");
        return FBA_ERR_UNSUPPORTED;
    }
    FBA_HIP(hipFuncSetAttribute((const void*)k_bwd_flow, hipFuncAttributeMaxDynamicSharedMemorySize, (int)BWD_LDS));
    // every level's trailing updates run inside the next level's k_panel (config 4: 968 iter/s merged
    // at any size vs 931 with the levels of > 450 tasks in their own k_syrk_multi launch, now that the
    // in-launch update runs on eight waves with coalesced whole-row loads; it measured the other way
    // round with the earlier four-wave sliced update)
    FBA_HIP(hipFuncSetAttribute((const void*)k_trtri128, hipFuncAttributeMaxDynamicSharedMemorySize, (int)TRTRI_LDS));

    // FBA_FLAG_SPINS (tests): the bound of every hand-off poll of THIS context (scal[SCAL_SPINS], read
    // by spin_expired), taken when the context is created; unset or <= 0: the default 1 << 22
    {
        const char* fs = getenv("FBA_FLAG_SPINS");
        const double v = spin_bound_value(fs ? atoll(fs) : 0);
        FBA_HIP(hipMemcpy(c.d_scal + SCAL_SPINS, &v, sizeof v, hipMemcpyHostToDevice));
    }
    c.probe_ev.assign(2 * std::max(c.sched.n_waves, 1), nullptr);
    for (auto& e : c.probe_ev) FBA_HIP(hipEventCreate(&e));
    return FBA_OK;
}

}  // namespace fba
