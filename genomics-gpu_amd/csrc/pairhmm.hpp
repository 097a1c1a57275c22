// pairhmm.hpp — PairHMM forward (fp32) as a segmented anti-diagonal wavefront.
//
// Reference recurrence: Non-CDP/PairHMM/inter_task/Synthetic_data/tile_1/tile_1.cu:44-177
// (identical arithmetic in Intra-task/.../improved_warp_based.cu:91-172).
// G lanes per pair, RR read rows per lane; haplotype bytes staged in LDS; the
// (M, I, D) of a lane's bottom row cross to the next lane with DPP wave_shr:1.
// The match/mismatch prior of a cell, (hb == rb) ? 1 - Qm : Qm / 3, is read from a
// per-lane LDS table indexed by the haplotype base (two ds_read_b128 per column
// for 8 rows, instead of 8 compares + 8 selects: 4,488 -> ~4,950 GCUPS on config
// 5, profiles/r02_pairhmm_ab.md); blocks with bases other than A/C/G/T compare.
// Every rounding step is the reference's: products and sums are separate
// roundings (__fmul_rn/__fadd_rn), the three FMAs are the reference's
// __fmaf_rn sites; this file is compiled with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace gx {

struct HmmArgs {
    const uint8_t *reads;
    const uint32_t *roff, *rlen;
    const float *qm, *delta, *xiksi, *alpha;
    const uint8_t *haps;
    const uint32_t *hoff, *hlen;
    float *result;
    uint32_t n;
    uint32_t lds_stride;   // bytes per pair slot (>= max haplotype length, multiple of 4)
    // QUALS kernels: Phred qualities per read base (at the read offsets) instead of
    // the four float parameters, mapped through the host's ph2pr table exactly as the
    // reference's host code does (tile_1.cu:216-220 table, :415-419 mapping)
    const uint8_t *bq, *iq, *dq;
    const float *ph2pr;    // 128 entries
    // length classes (dispatch.hip): this launch covers slots [slot0, n); slot -> pair
    // through perm (pairs sorted by read then haplotype length, tile_1.cu:180-195,325)
    const uint32_t *perm;
    uint32_t slot0;
};

// lane 0 of the wave reads 0 (bound_ctrl); no old value to set up
__device__ __forceinline__ float shr_lane_fb(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xF, 0xF, true));
}
__device__ __forceinline__ float shr_lane_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ bool acgt(uint32_t b) { return b == 'A' || b == 'C' || b == 'G' || b == 'T'; }
#ifndef GX_HMM_PKFMA
#define GX_HMM_PKFMA 0   // 1: the I and MM FMAs of a cell as one v_pk_fma_f32 (A/B: 4,574 vs 5,242 GCUPS, r03_pairhmm_ab.md)
#endif
#ifndef GX_HMM_PREFETCH
#define GX_HMM_PREFETCH 2   // 2: rows one column and bytes two ahead, fenced; 1: rows one column ahead, unfenced; 0: loaded in place
#endif
#ifndef GX_HMM_CODE16
#define GX_HMM_CODE16 0   // 1: the table path reads u16 table offsets per haplotype position (5,320 against 5,593: the extra LDS takes a block per CU)
#endif
#ifndef GX_HMM_MASKB
#define GX_HMM_MASKB 0   // 1: the table path's staged bytes masked to (hb & 6) once, one shift per column
#endif
#ifndef GX_HMM_WAVES
#define GX_HMM_WAVES 4   // waves per SIMD the register allocator must allow (4: 128 VGPRs + 16 B of scratch, 5,551 against 5,309 GCUPS at 3, profiles/r04/pairhmm_4w.json)
#endif
template <int G, int RR, bool QUALS = false, bool ABS = false>
__global__ __launch_bounds__(256, GX_HMM_WAVES) void pairhmm_kernel(HmmArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int P = 64 / G;
    const float c0 = 1.329228e+36f, c09 = 0.9f, c01 = 0.1f;     // tile_1.cu:228-233
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t lg = lane & (G - 1), slot = lane / G;
    const uint32_t idx = A.slot0 + (blockIdx.x * 4 + wave) * P + slot;
    const bool valid = idx < A.n;
    const uint32_t pair = (valid && A.perm) ? A.perm[idx] : idx;
    uint32_t R = 0, H = 0, ro = 0, ho = 0;
    if (valid) { R = A.rlen[pair]; H = A.hlen[pair]; ro = A.roff[pair]; ho = A.hoff[pair]; }

    // stage haplotypes; note whether the block holds a base other than A/C/G/T
    const uint32_t stride = A.lds_stride;
    uint8_t *wl = lds + (size_t)wave * P * stride;
    const uint32_t words = stride >> 2;
    bool other = false;
    for (uint32_t base = 0; base < P * words; base += 64) {
        const uint32_t idx = base + lane;
        const uint32_t ps = min(idx / words, (uint32_t)P - 1), w = idx - ps * words;
        const uint32_t pH = __shfl(H, ps * G), pho = __shfl(ho, ps * G);
        if (idx < P * words) {
            uint32_t v = 0;
            for (int b = 0; b < 4; ++b)
                if (4 * w + b < pH) {
                    const uint32_t hb = A.haps[pho + 4 * w + b];
                    other |= !acgt(hb);
                    v |= hb << (8 * b);
                }
            reinterpret_cast<uint32_t *>(wl + ps * stride)[w] = v;
        }
    }
    const uint8_t *hap = wl + slot * stride;

    // the lane's read rows and their parameters (tile_1.cu:89-118).  Rows are
    // bottom-aligned: the group covers rows [R - G*RR, R), so the read's last row
    // is always the bottom row of lane G-1 and the result sum needs no per-row
    // select.  The rows above row 0 are "virtual": prior 0, delta 0, xi 0 and D
    // decay 1.0, so from the boundary (M, I, D) = (0, 0, D0) they pass exactly
    // (0, 0, D0) down at every column.
    const int32_t r0 = (int32_t)(lg * RR) - (int32_t)(G * RR) + (int32_t)R;
    uint32_t rb[RR];
    float qm1[RR], qm3[RR], xi[RR], dk[RR];
    float Mk[RR], Dk[RR], MM[RR];
    // GX_HMM_PKFMA: (delta, alpha) of a row side by side, so the cell's two FMAs on MU
    // (I = MU*delta + I*0.1, MM = alpha*MU + 0.9*(I + D)) issue as one v_pk_fma_f32,
    // each element rounded as the scalar FMA (exact)
    typedef float hmf2 __attribute__((ext_vector_type(2)));
    hmf2 deal[RR];
    const float D0 = valid && H ? __fdiv_rn(c0, (float)H) : 0.f;      // constant[0]/(float)H
#pragma unroll
    for (int k = 0; k < RR; ++k) {
        const int32_t i = r0 + k;
        const bool in = valid && i >= 0;
        float q = 0.f, d = 0.f, x = 0.f, a = 0.f;
        if (in) {
            if (QUALS) {
                const uint32_t b = A.bq[ro + i] & 127u, iqv = A.iq[ro + i] & 127u, dqv = A.dq[ro + i] & 127u;
                q = A.ph2pr[b];
                d = A.ph2pr[iqv];
                x = A.ph2pr[dqv];
                a = __fsub_rn(1.0f, A.ph2pr[(iqv + dqv) & 127u]);
            } else {
                q = A.qm[ro + i]; d = A.delta[ro + i]; x = A.xiksi[ro + i]; a = A.alpha[ro + i];
            }
        }
        rb[k] = in ? A.reads[ro + i] : 0x100u;
        other |= in && !acgt(rb[k]);
        qm1[k] = in ? __fsub_rn(1.0f, q) : 0.f;     // Qm_1 = constant[1] - Qm
        qm3[k] = in ? __fdiv_rn(q, 3.0f) : 0.f;     // fdividef(Qm, 3) (<= 2 ulp in the reference)
        deal[k] = hmf2{d, a};
        xi[k] = x;
        dk[k] = in ? c01 : 1.0f;
        Mk[k] = 0.f;
        Dk[k] = in ? 0.f : D0;
        MM[k] = i == 0 ? __fmul_rn(c09, D0) : 0.f;                     // first row's MMID (:117)
    }
    // A/C/G/T blocks (every real input so far): the prior of each row for each
    // haplotype base, (hb == rb) ? 1 - Qm : Qm / 3, is tabulated once per lane in LDS,
    // so a column costs two 16-byte LDS reads instead of RR compares and selects.
    // Layout: [wave][code][quad][lane] float4, code = (base >> 1) & 3, so that the
    // lanes of one read are 16 consecutive bytes whatever their codes.
    const bool tab = !__syncthreads_or(other);
    constexpr int NQ = RR / 4;
    const uint32_t tbl_off = (4u * P * stride + 15u) & ~15u;
    const uint8_t *tb = lds + tbl_off + (size_t)wave * (4 * NQ * 64 * 16) + lane * 16;
    if (tab) {
        float4 *tw = reinterpret_cast<float4 *>(lds + tbl_off + (size_t)wave * (4 * NQ * 64 * 16) + lane * 16);
#pragma unroll
        for (int cd = 0; cd < 4; ++cd) {
            const uint32_t base = "ACTG"[cd];
#pragma unroll
            for (int qd = 0; qd < NQ; ++qd) {
                float v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = rb[4 * qd + u] == base ? qm1[4 * qd + u] : qm3[4 * qd + u];
                tw[(cd * NQ + qd) * 64] = make_float4(v[0], v[1], v[2], v[3]);
            }
        }
    }
#if GX_HMM_MASKB
    // table path: the staged bytes reduced to their code bits, (hb & 6), so a column's table
    // offset is one shift (this wave's own slots; the compare path keeps the bytes)
    if (tab) {
        for (uint32_t i = lane; i < P * stride; i += 64) wl[i] &= 6u;
        __builtin_amdgcn_wave_barrier();
    }
#endif
#if GX_HMM_CODE16
    // the table offset of every haplotype position, (hb & 6) * NQ * 512, as u16 after the
    // tables (one read and one add per column instead of a byte read, shift, mask and add)
    const uint32_t c16_off = tbl_off + 4u * (4 * NQ * 64 * 16);
    uint16_t *c16 = reinterpret_cast<uint16_t *>(lds + c16_off) + (size_t)wave * P * stride;
    if (tab) {
        for (uint32_t i = lane; i < P * stride; i += 64) c16[i] = (uint16_t)((wl[i] & 6u) * (NQ * 512u));
        __builtin_amdgcn_wave_barrier();
    }
    const uint16_t *hc16 = c16 + slot * stride;
#endif
    // rows' priors for haplotype byte hb: from the table (tab) or by compare
    auto tload = [&](uint32_t hb, float (&aa)[RR]) {
#if GX_HMM_CODE16
        const float4 *p = reinterpret_cast<const float4 *>(tb + hb);                         // hb: the u16 offset
#elif GX_HMM_MASKB
        const float4 *p = reinterpret_cast<const float4 *>(tb + hb * (NQ * 512u));          // hb = code bits
#else
        const float4 *p = reinterpret_cast<const float4 *>(tb + (hb & 6u) * (NQ * 512u));   // code * NQ * 1 KB
#endif
#pragma unroll
        for (int qd = 0; qd < NQ; ++qd) {
            const float4 x = p[qd * 64];
            aa[4 * qd] = x.x; aa[4 * qd + 1] = x.y; aa[4 * qd + 2] = x.z; aa[4 * qd + 3] = x.w;
        }
    };
    auto cload = [&](uint32_t hb, float (&aa)[RR]) {
#pragma unroll
        for (int k = 0; k < RR; ++k) aa[k] = (hb == rb[k]) ? qm1[k] : qm3[k];
    };

    // the sweep, instantiated once per prior source so that the compare path's
    // registers (rb, qm1, qm3) are dead in the table path
    const bool bottom = lg == G - 1;
    float acc = 0.f;
    // the table path's per-column source: u16 offsets (GX_HMM_CODE16) or haplotype bytes
    auto tsrc = [&](uint32_t j) -> uint32_t {
#if GX_HMM_CODE16
        return hc16[j];
#else
        return hap[j];
#endif
    };
    auto sweep = [&](auto tabc) {
        constexpr bool TABP = decltype(tabc)::value;
        uint32_t hmax = H;
    #pragma unroll
        for (int m = 32; m >= 1; m >>= 1) hmax = max(hmax, (uint32_t)__shfl_xor(hmax, m));
        const uint32_t nsteps = hmax + G - 1;
        float rM = 0.f, rI = 0.f, rD = 0.f;    // bottom-row values of the lane above, this column
        // ABS (every read of the launch shorter than G*RR rows, so row 0 of lane 0 is
        // virtual): that row takes I x 0 instead of I x 0.1, and with prior, delta and
        // alpha 0 and D decay 1 its outputs are (0, 0, D0) whatever finite (M, I, D)
        // comes in, so the top lane needs no boundary select in the steady steps
        const float c01_0 = (ABS && lg == 0) ? 0.f : c01;

        // one column j of the lane's rows; (MU, IU, DU) in = row r0-1, out = the lane's bottom row
        auto column = [&](const float (&aa)[RR], float &MU, float &IU, float &DU) {
    #pragma unroll
            for (int k = 0; k < RR; ++k) {
                const float MID = __fadd_rn(IU, DU);                   // :149-162
                const float DDM = __fmul_rn(Mk[k], xi[k]);
                const float IIMI = __fmul_rn(IU, k == 0 ? c01_0 : c01);
                const float MIIDD = __fmul_rn(c09, MID);
                const float Mn = __fmul_rn(aa[k], MM[k]);
#if GX_HMM_PKFMA
                const hmf2 im = __builtin_elementwise_fma(hmf2{MU, MU}, deal[k], hmf2{IIMI, MIIDD});
                const float In = im.x;
                const float Dn = __fmaf_rn(Dk[k], dk[k], DDM);
                MM[k] = im.y;
#else
                const float In = __fmaf_rn(MU, deal[k].x, IIMI);
                const float Dn = __fmaf_rn(Dk[k], dk[k], DDM);
                MM[k] = __fmaf_rn(deal[k].y, MU, MIIDD);
#endif
                Mk[k] = Mn; Dk[k] = Dn;
                MU = Mn; IU = In; DU = Dn;
            }
        };
        auto checked_step = [&](uint32_t s) {
            const int32_t j = (int32_t)s - (int32_t)lg;
            float MU, IU, DU;
            if (lg == 0) { MU = 0.f; IU = 0.f; DU = D0; }                  // row -1: M=I=0, D=D0
            else { MU = rM; IU = rI; DU = rD; }
            if (valid && j >= 0 && (uint32_t)j < H) {
                float aa[RR];
                if constexpr (TABP) tload(tsrc(j), aa);
                else cload(hap[j], aa);
                column(aa, MU, IU, DU);
                if (bottom) acc = __fadd_rn(acc, __fadd_rn(MU, IU));       // row R-1, column j (:166-167)
            }
            rM = shr_lane_f(MU); rI = shr_lane_f(IU); rD = shr_lane_f(DU);
        };
        // steps [G-1, hmin): every lane of the wave is inside its pair's columns, so
        // no activity test and no merge of state
        auto steady = [&](const float (&aa)[RR]) {
            float MU = rM, IU = rI, DU = rD;
            if (!ABS && lg == 0) { MU = 0.f; IU = 0.f; DU = D0; }
            column(aa, MU, IU, DU);
            acc = __fadd_rn(acc, __fadd_rn(MU, IU));                       // kept by the bottom lane only
            if constexpr (ABS) { rM = shr_lane_fb(MU); rI = shr_lane_fb(IU); rD = shr_lane_fb(DU); }
            else { rM = shr_lane_f(MU); rI = shr_lane_f(IU); rD = shr_lane_f(DU); }
        };
        {
            uint32_t hmin = valid ? H : 0u;
    #pragma unroll
            for (int m = 32; m >= 1; m >>= 1) hmin = min(hmin, (uint32_t)__shfl_xor(hmin, m));
            const uint32_t s1 = min((uint32_t)G - 1, nsteps), s2 = max(s1, hmin);
            for (uint32_t s = 0; s < s1; ++s) checked_step(s);
            if constexpr (TABP && !GX_HMM_PREFETCH) {
                // one register set: each column's table rows loaded where the column starts
                // (8 VGPRs fewer; the other waves of the SIMD cover the LDS latency)
                for (uint32_t s = s1; s < hmin; ++s) {
                    float aa[RR];
                    tload(tsrc(s - lg), aa);
                    steady(aa);
                }
            } else if constexpr (TABP && GX_HMM_PREFETCH == 2) {
                // table rows one column ahead and haplotype bytes two ahead, pinned in place
                // by scheduling fences: left to itself the scheduler sinks the loads next to
                // their first use (the row read then waits on the byte read, and the column on
                // the row read).  Loop bounds are wave-uniform (SGPR loop).  Byte reads past a
                // pair's columns (up to column hmin + 1) stay inside the slot + table region
                // and are not used.
                const uint32_t he = __builtin_amdgcn_readfirstlane(hmin);
                float aaA[RR], aaB[RR];
                uint32_t s = __builtin_amdgcn_readfirstlane(s1);
                uint32_t hbn = 0;
                if (s < he) { tload(tsrc(s - lg), aaA); hbn = tsrc(s + 1 - lg); }
                for (; s + 1 < he; s += 2) {
                    tload(hbn, aaB);
                    hbn = tsrc(s + 2 - lg);
                    __builtin_amdgcn_sched_barrier(0);
                    steady(aaA);
                    __builtin_amdgcn_sched_barrier(0);
                    tload(hbn, aaA);
                    hbn = tsrc(s + 3 - lg);
                    __builtin_amdgcn_sched_barrier(0);
                    steady(aaB);
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (s < he) steady(aaA);
            } else if constexpr (TABP) {
                // table rows one step ahead, two register sets in turn (hap reads past a
                // pair's columns stay inside the slot + table region and are not used)
                float aaA[RR], aaB[RR];
                uint32_t s = s1;
                if (s < hmin) tload(tsrc(s - lg), aaA);
                for (; s + 1 < hmin; s += 2) {
                    tload(tsrc(s + 1 - lg), aaB);
                    steady(aaA);
                    tload(tsrc(s + 2 - lg), aaA);
                    steady(aaB);
                }
                if (s < hmin) steady(aaA);
            } else {
                for (uint32_t s = s1; s < hmin; ++s) {
                    float aa[RR];
                    cload(hap[s - lg], aa);
                    steady(aa);
                }
            }
            for (uint32_t s = s2; s < nsteps; ++s) checked_step(s);
        }
    };
    if (tab) sweep(std::true_type{});
    else sweep(std::false_type{});
    if (valid && bottom) A.result[pair] = acc;
}


// ---------------------------------------------------------------------------
// Two problems per lane group (pairhmm2_kernel): slots 2s and 2s + 1 of the launch run
// in the two elements of float2 registers, so the three FMAs of a cell pair issue as
// v_pk_fma_f32 (4.6 cycles for two, against 4.1 each for v_fmac_f32 on gfx950,
// profiles/r02_ubench_hmm.txt), the add and the products as v_pk_add / v_pk_mul.  The
// prior x MM product reads a per-problem table row, so it stays two v_mul_f32.  Every
// element op is the scalar kernel's (same roundings, same order): results are bit-equal
// to pairhmm_kernel.  Rows, boundaries and phases as pairhmm_kernel; steps where an
// element is outside its problem's columns (different haplotype lengths) commit per
// element.
// ---------------------------------------------------------------------------
typedef float hf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ hf2 hfma2(hf2 a, hf2 b, hf2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ hf2 shr_lane_f2(hf2 v) { return hf2{shr_lane_f(v.x), shr_lane_f(v.y)}; }
__device__ __forceinline__ hf2 shr_lane_fb2(hf2 v) { return hf2{shr_lane_fb(v.x), shr_lane_fb(v.y)}; }

#ifndef GX_HMM2_WAVES
#define GX_HMM2_WAVES 2
#endif
template <int G, int RR, bool QUALS = false, bool ABS = false>
__global__ __launch_bounds__(256, RR <= 4 ? 3 : GX_HMM2_WAVES) void pairhmm2_kernel(HmmArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int P = 64 / G;              // lane groups per wave, two problems each
    const float c0 = 1.329228e+36f, c09 = 0.9f, c01 = 0.1f;     // tile_1.cu:228-233
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t lg = lane & (G - 1), slot = lane / G;
    bool valid[2];
    uint32_t pair[2], R[2], H[2], ro[2], ho[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t idx = A.slot0 + (blockIdx.x * 4 + wave) * (2 * P) + 2 * slot + h;
        valid[h] = idx < A.n;
        pair[h] = (valid[h] && A.perm) ? A.perm[idx] : idx;
        R[h] = H[h] = ro[h] = ho[h] = 0;
        if (valid[h]) { R[h] = A.rlen[pair[h]]; H[h] = A.hlen[pair[h]]; ro[h] = A.roff[pair[h]]; ho[h] = A.hoff[pair[h]]; }
    }

    // stage the wave's 2P haplotypes; note whether the block holds a base other than A/C/G/T
    const uint32_t stride = A.lds_stride;
    uint8_t *wl = lds + (size_t)wave * 2 * P * stride;
    const uint32_t words = stride >> 2;
    bool other = false;
    for (uint32_t base = 0; base < 2 * P * words; base += 64) {
        const uint32_t i = base + lane;
        const uint32_t q = min(i / words, (uint32_t)(2 * P) - 1), w = i - q * words;
        const uint32_t src = (q >> 1) * G;   // the first lane of problem q's group
        const uint32_t pH0 = __shfl(H[0], src), pH1 = __shfl(H[1], src);
        const uint32_t ph0 = __shfl(ho[0], src), ph1 = __shfl(ho[1], src);
        const uint32_t pH = (q & 1) ? pH1 : pH0, pho = (q & 1) ? ph1 : ph0;
        if (i < 2 * P * words) {
            uint32_t v = 0;
            for (int b = 0; b < 4; ++b)
                if (4 * w + b < pH) {
                    const uint32_t hb = A.haps[pho + 4 * w + b];
                    other |= !acgt(hb);
                    v |= hb << (8 * b);
                }
            reinterpret_cast<uint32_t *>(wl + q * stride)[w] = v;
        }
    }
    const uint8_t *hapA = wl + (2 * slot) * stride, *hapB = hapA + stride;

    // rows (bottom-aligned per problem, as pairhmm_kernel)
    uint32_t rb[2][RR];
    hf2 qm1[RR], qm3[RR], de[RR], xi[RR], al[RR], dk[RR], Mk[RR], Dk[RR], MM[RR];
    hf2 D0;
#pragma unroll
    for (int h = 0; h < 2; ++h) D0[h] = valid[h] && H[h] ? __fdiv_rn(c0, (float)H[h]) : 0.f;
#pragma unroll
    for (int k = 0; k < RR; ++k) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int32_t i = (int32_t)(lg * RR) - (int32_t)(G * RR) + (int32_t)R[h] + k;
            const bool in = valid[h] && i >= 0;
            float q = 0.f, d = 0.f, x = 0.f, a = 0.f;
            if (in) {
                if (QUALS) {
                    const uint32_t b = A.bq[ro[h] + i] & 127u, iqv = A.iq[ro[h] + i] & 127u, dqv = A.dq[ro[h] + i] & 127u;
                    q = A.ph2pr[b];
                    d = A.ph2pr[iqv];
                    x = A.ph2pr[dqv];
                    a = __fsub_rn(1.0f, A.ph2pr[(iqv + dqv) & 127u]);
                } else {
                    q = A.qm[ro[h] + i]; d = A.delta[ro[h] + i]; x = A.xiksi[ro[h] + i]; a = A.alpha[ro[h] + i];
                }
            }
            rb[h][k] = in ? A.reads[ro[h] + i] : 0x100u;
            other |= in && !acgt(rb[h][k]);
            qm1[k][h] = in ? __fsub_rn(1.0f, q) : 0.f;
            qm3[k][h] = in ? __fdiv_rn(q, 3.0f) : 0.f;
            de[k][h] = d;
            xi[k][h] = x;
            al[k][h] = a;
            dk[k][h] = in ? c01 : 1.0f;
            Mk[k][h] = 0.f;
            Dk[k][h] = in ? 0.f : D0[h];
            MM[k][h] = i == 0 ? __fmul_rn(c09, D0[h]) : 0.f;
        }
    }
    // per-problem prior tables: [wave][problem][code][quad][lane] float4
    const bool tab = !__syncthreads_or(other);
    constexpr int NQ = RR / 4;
    constexpr uint32_t TBL = 4 * NQ * 64 * 16;          // bytes of one problem's table per wave
    const uint32_t tbl_off = (4u * 2 * P * stride + 15u) & ~15u;
    const uint8_t *tbA = lds + tbl_off + (size_t)wave * 2 * TBL + lane * 16, *tbB = tbA + TBL;
    if (tab) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float4 *tw = reinterpret_cast<float4 *>(lds + tbl_off + (size_t)wave * 2 * TBL + h * TBL + lane * 16);
#pragma unroll
            for (int cd = 0; cd < 4; ++cd) {
                const uint32_t base = "ACTG"[cd];
#pragma unroll
                for (int qd = 0; qd < NQ; ++qd) {
                    float v[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        v[u] = rb[h][4 * qd + u] == base ? qm1[4 * qd + u][h] : qm3[4 * qd + u][h];
                    tw[(cd * NQ + qd) * 64] = make_float4(v[0], v[1], v[2], v[3]);
                }
            }
        }
    }
    // rows' priors of column j of each problem: aa[h][k]
    auto tload = [&](uint32_t hbA, uint32_t hbB, float (&aa)[2][RR]) {
        const float4 *pa = reinterpret_cast<const float4 *>(tbA + (hbA & 6u) * (NQ * 512u));
        const float4 *pb = reinterpret_cast<const float4 *>(tbB + (hbB & 6u) * (NQ * 512u));
#pragma unroll
        for (int qd = 0; qd < NQ; ++qd) {
            const float4 x = pa[qd * 64], y = pb[qd * 64];
            aa[0][4 * qd] = x.x; aa[0][4 * qd + 1] = x.y; aa[0][4 * qd + 2] = x.z; aa[0][4 * qd + 3] = x.w;
            aa[1][4 * qd] = y.x; aa[1][4 * qd + 1] = y.y; aa[1][4 * qd + 2] = y.z; aa[1][4 * qd + 3] = y.w;
        }
    };
    auto cload = [&](uint32_t hbA, uint32_t hbB, float (&aa)[2][RR]) {
#pragma unroll
        for (int k = 0; k < RR; ++k) {
            aa[0][k] = (hbA == rb[0][k]) ? qm1[k][0] : qm3[k][0];
            aa[1][k] = (hbB == rb[1][k]) ? qm1[k][1] : qm3[k][1];
        }
    };

    const bool bottom = lg == G - 1;
    hf2 acc = {0.f, 0.f};
    auto sweep = [&](auto tabc) {
        constexpr bool TABP = decltype(tabc)::value;
        uint32_t hmax = max(H[0], H[1]);
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) hmax = max(hmax, (uint32_t)__shfl_xor(hmax, m));
        const uint32_t nsteps = hmax + G - 1;
        hf2 rM = {0.f, 0.f}, rI = {0.f, 0.f}, rD = {0.f, 0.f};
        const float c01_0 = (ABS && lg == 0) ? 0.f : c01;
        const hf2 C09 = {c09, c09};

        // one column of the lane's rows for both problems; MASK: commit element h only where act[h]
        auto column = [&](const float (&aa)[2][RR], hf2 &MU, hf2 &IU, hf2 &DU, auto maskc, const bool (&act)[2]) {
            constexpr bool MASK = decltype(maskc)::value;
#pragma unroll
            for (int k = 0; k < RR; ++k) {
                const hf2 MID = IU + DU;                               // :149-162, per element
                const hf2 DDM = Mk[k] * xi[k];
                const float ci = k == 0 ? c01_0 : c01;
                const hf2 IIMI = IU * hf2{ci, ci};
                const hf2 MIIDD = C09 * MID;
                hf2 Mn;
                Mn.x = __fmul_rn(aa[0][k], MM[k].x);
                Mn.y = __fmul_rn(aa[1][k], MM[k].y);
                const hf2 In = hfma2(MU, de[k], IIMI);
                const hf2 Dn = hfma2(Dk[k], dk[k], DDM);
                const hf2 MMn = hfma2(al[k], MU, MIIDD);
                if constexpr (MASK) {
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        if (act[h]) { MM[k][h] = MMn[h]; Mk[k][h] = Mn[h]; Dk[k][h] = Dn[h]; MU[h] = Mn[h]; IU[h] = In[h]; DU[h] = Dn[h]; }
                    }
                } else {
                    MM[k] = MMn; Mk[k] = Mn; Dk[k] = Dn;
                    MU = Mn; IU = In; DU = Dn;
                }
            }
        };
        auto checked_step = [&](uint32_t s) {
            const int32_t j = (int32_t)s - (int32_t)lg;
            hf2 MU, IU, DU;
            if (lg == 0) { MU = hf2{0.f, 0.f}; IU = hf2{0.f, 0.f}; DU = D0; }  // row -1: M=I=0, D=D0
            else { MU = rM; IU = rI; DU = rD; }
            bool act[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) act[h] = valid[h] && j >= 0 && (uint32_t)j < H[h];
            if (act[0] || act[1]) {
                float aa[2][RR];
                const uint32_t hbA = hapA[act[0] ? j : 0], hbB = hapB[act[1] ? j : 0];
                if constexpr (TABP) tload(hbA, hbB, aa);
                else cload(hbA, hbB, aa);
                if (act[0] && act[1]) column(aa, MU, IU, DU, std::false_type{}, act);
                else column(aa, MU, IU, DU, std::true_type{}, act);
                if (bottom) {
                    const hf2 t = acc + (MU + IU);                        // row R-1, column j (:166-167)
                    if (act[0]) acc.x = t.x;
                    if (act[1]) acc.y = t.y;
                }
            }
            rM = shr_lane_f2(MU); rI = shr_lane_f2(IU); rD = shr_lane_f2(DU);
        };
        const bool none[2] = {false, false};
        auto steady = [&](const float (&aa)[2][RR]) {
            hf2 MU = rM, IU = rI, DU = rD;
            if (!ABS && lg == 0) { MU = hf2{0.f, 0.f}; IU = hf2{0.f, 0.f}; DU = D0; }
            column(aa, MU, IU, DU, std::false_type{}, none);
            acc = acc + (MU + IU);                                        // kept by the bottom lane only
            if constexpr (ABS) { rM = shr_lane_fb2(MU); rI = shr_lane_fb2(IU); rD = shr_lane_fb2(DU); }
            else { rM = shr_lane_f2(MU); rI = shr_lane_f2(IU); rD = shr_lane_f2(DU); }
        };
        {
            uint32_t hmin = min(valid[0] ? H[0] : 0u, valid[1] ? H[1] : 0u);
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) hmin = min(hmin, (uint32_t)__shfl_xor(hmin, m));
            const uint32_t s1 = min((uint32_t)G - 1, nsteps), s2 = max(s1, hmin);
            for (uint32_t s = 0; s < s1; ++s) checked_step(s);
            if constexpr (TABP) {
                float aaA[2][RR], aaB[2][RR];
                uint32_t s = s1;
                if (s < hmin) tload(hapA[s - lg], hapB[s - lg], aaA);
                for (; s + 1 < hmin; s += 2) {
                    tload(hapA[s + 1 - lg], hapB[s + 1 - lg], aaB);
                    steady(aaA);
                    tload(hapA[s + 2 - lg], hapB[s + 2 - lg], aaA);
                    steady(aaB);
                }
                if (s < hmin) steady(aaA);
            } else {
                for (uint32_t s = s1; s < hmin; ++s) {
                    float aa[2][RR];
                    cload(hapA[s - lg], hapB[s - lg], aa);
                    steady(aa);
                }
            }
            for (uint32_t s = s2; s < nsteps; ++s) checked_step(s);
        }
    };
    if (tab) sweep(std::true_type{});
    else sweep(std::false_type{});
#pragma unroll
    for (int h = 0; h < 2; ++h)
        if (valid[h] && bottom) A.result[pair[h]] = acc[h];
}

}  // namespace gx
