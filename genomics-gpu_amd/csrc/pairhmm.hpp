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
// waves per SIMD the register allocator must allow (4: 128 VGPRs + 16 B of scratch, 5,551 against
// 5,309 GCUPS at 3, profiles/r04/pairhmm_4w.json)
constexpr int kHmmWaves = 4;
template <int G, int RR, bool QUALS = false, bool ABS = false>
__global__ __launch_bounds__(256, kHmmWaves) void pairhmm_kernel(HmmArgs A) {
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
    // (delta, alpha) of a row
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
    // rows' priors for haplotype byte hb: from the table (tab) or by compare
    auto tload = [&](uint32_t hb, float (&aa)[RR]) {
        const float4 *p = reinterpret_cast<const float4 *>(tb + (hb & 6u) * (NQ * 512u));   // code * NQ * 1 KB
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
    // the table path's per-column source: the haplotype bytes
    auto tsrc = [&](uint32_t j) -> uint32_t {
        return hap[j];
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
                const float In = __fmaf_rn(MU, deal[k].x, IIMI);
                const float Dn = __fmaf_rn(Dk[k], dk[k], DDM);
                MM[k] = __fmaf_rn(deal[k].y, MU, MIIDD);
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
            if constexpr (TABP) {
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


}  // namespace gx
