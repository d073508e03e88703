// SBR (HE-AAC v1) signal path for gfx950: QMF analysis -> HF generation -> HF adjustment -> QMF
// synthesis -> PCM, one wave per (chunk of frames, channel).  A/ = aac/src/main/java/net/
// sourceforge/jaad/aac/ of the reference; every binary32 expression keeps the Java evaluation
// order (the library is built with -ffp-contract=off), so the output is bit-identical to the
// oracle's restatement.
//
// Lane roles (64-wide wave):
//   * band phases: lane k = QMF band k; the Xsbr matrix of the channel (40 rows) lives in
//     80 VGPRs of that lane, so HF generation, envelope estimation and assembly are lane-local
//     except for the patch source, fetched with ds_bpermute;
//   * DCT-IV phases (A/sbr/DCT.java): a 32-point DCT-IV is spread over 32 lanes (one complex
//     point per lane); the radix-2 DIF stages exchange partners with ds_swizzle (xor 16..1).
//     Analysis runs two slots per pass (lanes 0-31 / 32-63), synthesis runs the two DCTs of
//     one slot per pass;
//   * synthesis window: lane k = output sample 64*l + k, reading a 10-slot ring of v blocks in LDS.
#include <hip/hip_runtime.h>

#include "jaad_sbr.h"

namespace jaad {
namespace {

constexpr int kWin = 1312 + 1312 / 32 + 8;  // analysis window, padded one float per 32
__device__ __forceinline__ int wp(int i) { return i + (i >> 5); }

struct SbrLds {
    float win[kWin];
    float vring[10][128];
    float ecurr[5][64];
    float gl[5][64], ql[5][64], sl[5][64];
    float gq_eo[64], gq_qm[64], gq_sm[64], gq_g[64];  // per-envelope gain inputs
};

__device__ __forceinline__ int lane_id() { return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

template <int kXor>
__device__ __forceinline__ float swz(float v)
{
    return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x1F | (kXor << 10)));
}
__device__ __forceinline__ float shfl(float v, int src_lane)
{
    return __int_as_float(__builtin_amdgcn_ds_bpermute(src_lane << 2, __float_as_int(v)));
}

// Math.round + short clamp (S/SampleBuffer.java:190-205)
__device__ __forceinline__ int java_round16(float s)
{
    if (s != s) return 0;
    const float fl = floorf(s);
    int r = (s - fl) >= 0.5f ? (int)fl + 1 : (int)fl;
    if (s >= 2147483648.0f) r = 2147483647;
    if (s <= -2147483648.0f) r = (int)0x80000000;
    return r > 32767 ? 32767 : (r < -32768 ? -32768 : r);
}

__device__ __forceinline__ float java_minf(float a, float b)
{
    if (a != a) return a;
    if (a == 0.0f && b == 0.0f) return __float_as_uint(a) >> 31 ? a : b;
    return a <= b ? a : b;
}

// per-lane constants of a 32-point DCT-IV element e (A/sbr/DCT.java:347-391)
struct DctConst {
    float t0, t32, t64;        // pre-modulation
    float t96, t128, t160;     // post-modulation
    float w1r, w1i, w2r, w2i;  // stage 1/2 twiddles of the bottom lanes
    float w3;                  // stage 3 constant (w[4] or w[12])
};

// DCT.dct4_kernel distributed over the 32 lanes of a half-wave: (xr, xi) = input element e,
// returns output element e.  Each stage performs, per element, exactly the operation the
// sequential Java loop performs on it.
__device__ __forceinline__ void dct4(const DctConst& K, int e, int half_base, float xr, float xi, float& orr,
                                     float& oi)
{
    float tmp = (xr + xi) * K.t0;
    float r = (xi * K.t64) + tmp;
    float i = (xr * K.t32) + tmp;
    // stage 1 (DCT.java:143-164): pairs (i, i+16)
    {
        const float pr = swz<16>(r), pi = swz<16>(i);
        if (e < 16) {
            r = r + pr;
            i = i + pi;
        } else {
            const float tr = pr - r, ti = pi - i;
            r = (tr * K.w1r) - (ti * K.w1i);
            i = (tr * K.w1i) + (ti * K.w1r);
        }
    }
    // stage 2 (:166-207): pairs (i, i+8) in each 16-group, twiddle w[2j]
    {
        const float pr = swz<8>(r), pi = swz<8>(i);
        if (!(e & 8)) {
            r = r + pr;
            i = i + pi;
        } else {
            const float tr = pr - r, ti = pi - i;
            r = (tr * K.w2r) - (ti * K.w2i);
            i = (tr * K.w2i) + (ti * K.w2r);
        }
    }
    // stage 3 (:212-287): pairs (i, i+4) in each 8-group; four bottom variants
    {
        const float pr = swz<4>(r), pi = swz<4>(i);
        if (!(e & 4)) {
            r = r + pr;
            i = i + pi;
        } else {
            const int v = e & 3;
            const float tr = pr - r, ti = pi - i;
            if (v == 0) {
                r = tr;
                i = ti;
            } else if (v == 1) {
                const float a = tr + ti, b = ti - tr;
                r = a * K.w3;
                i = b * K.w3;
            } else if (v == 2) {
                const float nr = ti, ni = r - pr;
                r = nr;
                i = ni;
            } else {
                const float a = tr - ti, b = tr + ti;
                r = a * K.w3;
                i = b * K.w3;
            }
        }
    }
    // stage 4 (:291-322): pairs (i, i+2) in each 4-group
    {
        const float pr = swz<2>(r), pi = swz<2>(i);
        if (!(e & 2)) {
            r = r + pr;
            i = i + pi;
        } else if (!(e & 1)) {
            r = pr - r;
            i = pi - i;
        } else {
            const float nr = pi - i, ni = r - pr;
            r = nr;
            i = ni;
        }
    }
    // stage 5 (:326-341): pairs (i, i+1)
    {
        const float pr = swz<1>(r), pi = swz<1>(i);
        if (!(e & 1)) {
            r = r + pr;
            i = i + pi;
        } else {
            r = pr - r;
            i = pi - i;
        }
    }
    // post-modulation with bit-reversed reads (:368-389)
    const int br = (int)(__builtin_bitreverse32((uint32_t)e) >> 27);
    const float x_re = shfl(r, half_base + br), x_im = shfl(i, half_base + br);
    if (e == 16) {
        orr = (x_re + x_im) * K.t96;
        oi = (x_im - x_re) * K.t96;
    } else {
        const float t = (x_re + x_im) * K.t96;
        orr = (x_im * K.t160) + t;
        oi = (x_re * K.t128) + t;
    }
}

__global__ __launch_bounds__(64, 1) void sbr_kernel(SbrArgs A)
{
    __shared__ SbrLds L;
    const SbrChunk ck = A.chunks[blockIdx.x];
    const int u = lane_id();
    const int e = u & 31, half = u >> 5, hb = half << 5;
    const int c = ck.ch;
    const int nch = A.nch;

    // ---- lane constants ----
    DctConst K;
    {
        const float* t = A.dct;
        const float* wr = A.dct + 192;
        const float* wi = A.dct + 208;
        K.t0 = t[e];
        K.t32 = t[e + 32];
        K.t64 = t[e + 64];
        K.t96 = t[e + 96];
        K.t128 = t[e + 128];
        K.t160 = t[e + 160];
        K.w1r = wr[e & 15];
        K.w1i = wi[e & 15];
        K.w2r = wr[2 * (e & 7)];
        K.w2i = wi[2 * (e & 7)];
        K.w3 = (e & 3) == 1 ? wr[4] : wr[12];
    }
    float ca[5], cb[5], cw[10];
#pragma unroll
    for (int j = 0; j < 5; j++) {
        ca[j] = A.qmf_c[2 * (e + 64 * j)];
        cb[j] = A.qmf_c[2 * (e + 32 + 64 * j)];
    }
#pragma unroll
    for (int t = 0; t < 10; t++) cw[t] = A.qmf_c[u + 64 * t];
    const float rel = __fdiv_rn(1.0f, 1.0f + 1e-6f);

    // ---- channel state ----
    float xr[40], xi[40];
    float gr[5], qr[5];
    int gidx = 0;   // GQ_ringbuf_index
    int vpos = 0;   // next v-ring slot
#pragma unroll
    for (int r = 0; r < 40; r++) xr[r] = xi[r] = 0.0f;
#pragma unroll
    for (int j = 0; j < 5; j++) gr[j] = qr[j] = 0.0f;
    for (int i = u; i < 10 * 128; i += 64) (&L.vring[0][0])[i] = 0.0f;

    const float* tail_src = nullptr;  // last 288 samples before the current frame
    if (ck.flags & kSbrChunkLoad) {
        const SbrChState& S = A.state_in[(size_t)ck.slot * 2 + c];
#pragma unroll
        for (int r = 0; r < 8; r++) {
            xr[r] = S.carry[r][u][0];
            xi[r] = S.carry[r][u][1];
        }
        for (int i = u; i < 9 * 128; i += 64) (&L.vring[1][0])[i] = (&S.vhist[0][0])[i];  // slots 1..9
        vpos = 0;  // ring[1..9] = history oldest..newest? see below
#pragma unroll
        for (int j = 0; j < 5; j++) {
            gr[j] = S.gq[0][j][u];
            qr[j] = S.gq[1][j][u];
        }
        gidx = (int)S.gq_index;
        tail_src = S.tail;
    }
    // history layout: vring[(vpos - 1 - j) mod 10] = slot (current-1-j); vhist[8] is the newest.
    // After the load above ring[1..9] = vhist[0..8] (oldest .. newest), so the newest is ring[9]
    // and the next slot goes to ring[0]: vpos = 0 -> ring[(0-1) mod 10] = ring[9]. Consistent.

    auto load_window = [&](const float* tail, const float* cur) {
        for (int i = u; i < 288; i += 64) L.win[wp(i)] = tail ? tail[i] : 0.0f;
        for (int i = u; i < 1024; i += 64) L.win[wp(288 + i)] = cur[i];
        __syncthreads();
    };

    // AnalysisFilterbank.sbr_qmf_analysis_32 for slots [2*p0, 2*p1) into rows 8 + slot
    auto analysis = [&](int p0, int kx) {
#pragma unroll
        for (int p = 0; p < 16; p++) {
            if (p < p0) continue;
            const int base = 288 + 32 * (2 * p + half) + 31;
            float ulo, uhi;
            {
                const float a0 = L.win[wp(base - e)] * ca[0], a1 = L.win[wp(base - e - 64)] * ca[1];
                const float a2 = L.win[wp(base - e - 128)] * ca[2], a3 = L.win[wp(base - e - 192)] * ca[3];
                const float a4 = L.win[wp(base - e - 256)] * ca[4];
                ulo = (((a0 + a1) + a2) + a3) + a4;
                const int n = e + 32;
                const float b0 = L.win[wp(base - n)] * cb[0], b1 = L.win[wp(base - n - 64)] * cb[1];
                const float b2 = L.win[wp(base - n - 128)] * cb[2], b3 = L.win[wp(base - n - 192)] * cb[3];
                const float b4 = L.win[wp(base - n - 256)] * cb[4];
                uhi = (((b0 + b1) + b2) + b3) + b4;
            }
            // in_real[0] = u[0], in_real[n] = -u[64-n]; in_imag[m] = u[32-m]  (:39-46)
            const int src = hb + ((32 - e) & 31);
            const float slo = shfl(ulo, src), shi = shfl(uhi, src);
            const float in_r = e == 0 ? ulo : -shi;
            const float in_i = e == 0 ? uhi : slo;
            float orr, oi;
            dct4(K, e, hb, in_r, in_i, orr, oi);
            // X[2n] = 2*out[n], X[2n+1] = -2*swap(out[31-n])  (:52-71); band lane k reads its slot
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const int k = u;
                const int srcl = 32 * s + ((k & 1) ? 31 - (k >> 1) : (k >> 1));
                const float vr = shfl(orr, srcl & 63), vi = shfl(oi, srcl & 63);
                float re = 0.0f, im = 0.0f;
                if (k < kx && k < 32) {
                    if (k & 1) {
                        re = -2.0f * vi;
                        im = -2.0f * vr;
                    } else {
                        re = 2.0f * vr;
                        im = 2.0f * vi;
                    }
                }
                xr[8 + 2 * p + s] = re;
                xi[8 + 2 * p + s] = im;
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    auto carry_shift = [&]() {  // SBR.sbr_save_matrix (A/sbr/SBR.java:286-300)
#pragma unroll
        for (int r = 0; r < 8; r++) {
            xr[r] = xr[r + 32];
            xi[r] = xi[r + 32];
        }
#pragma unroll
        for (int r = 8; r < 40; r++) xr[r] = xi[r] = 0.0f;
    };

    auto process = [&](int f, const float* tail, bool emit) {
        const size_t cf = (size_t)f * nch + c;
        const SbrRec& R = A.recs[cf];
        const SbrTab& T = A.tabs[R.table];
        const int kx = T.kx, M = T.M, L_E = R.L_E;
        const int first = R.t_E[0], last = R.t_E[L_E];
        const int s_lim = R.lim_bands;
        load_window(tail, A.time + cf * 1024);
        analysis(0, kx);
        __syncthreads();

        // ---------- HF generation (A/sbr/HFGeneration.java:17-98, 100-196) ----------
        float a0r = 0, a0i = 0, a1r = 0, a1i = 0;
        {
            float r01r = 0, r01i = 0, r02r = 0, r02i = 0, r11r = 0;
            float t1r, t1i, t2r = xr[0], t2i = xi[0], t3r = xr[1], t3i = xi[1];
            const float t4r = t2r, t4i = t2i, t5r = t3r, t5i = t3i;
#pragma unroll
            for (int j = 2; j < 40; j++) {
                t1r = t2r;
                t1i = t2i;
                t2r = t3r;
                t2i = t3i;
                t3r = xr[j];
                t3i = xi[j];
                r01r += t3r * t2r + t3i * t2i;
                r01i += t3i * t2r - t3r * t2i;
                r02r += t3r * t1r + t3i * t1i;
                r02i += t3i * t1r - t3r * t1i;
                r11r += t2r * t2r + t2i * t2i;
            }
            const float r12r = r01r - (t3r * t2r + t3i * t2i) + (t5r * t4r + t5i * t4i);
            const float r12i = r01i - (t3i * t2r - t3r * t2i) + (t5i * t4r - t5r * t4i);
            const float r22r = r11r - (t2r * t2r + t2i * t2i) + (t4r * t4r + t4i * t4i);
            const float det = (r11r * r22r) - (rel * ((r12r * r12r) + (r12i * r12i)));
            if (det != 0.0f) {
                const float tmp = __fdiv_rn(1.0f, det);
                a1r = ((r01r * r12r) - (r01i * r12i) - (r02r * r11r)) * tmp;
                a1i = ((r01i * r12r) + (r01r * r12i) - (r02i * r11r)) * tmp;
            }
            if (r11r != 0.0f) {
                const float tmp = __fdiv_rn(1.0f, r11r);
                a0r = -(r01r + (a1r * r12r) + (a1i * r12i)) * tmp;
                a0i = -(r01i + (a1i * r12r) - (a1r * r12i)) * tmp;
            }
            if (((a0r * a0r) + (a0i * a0i) >= 16.0f) || ((a1r * a1r) + (a1i * a1i) >= 16.0f)) a0r = a0i = a1r = a1i = 0.0f;
        }
        {
            const int p = T.src_p[u];
            const bool gen = p != 0xFF;
            const int ps = gen ? p : u;
            const float bw = R.bw[T.g_of_k[u] < 5 ? T.g_of_k[u] : 0];
            const float bw2 = bw * bw;
            const float A0r = shfl(a0r, ps) * bw, A1r = shfl(a1r, ps) * bw2;
            const float A0i = shfl(a0i, ps) * bw, A1i = shfl(a1i, ps) * bw2;
            float p1r = 0, p1i = 0, p2r = 0, p2i = 0;  // source rows r-2, r-1
#pragma unroll
            for (int r = 0; r < 40; r++) {
                const float sr = shfl(xr[r], ps), si = shfl(xi[r], ps);
                const int l = r - 2;
                if (gen && l >= first && l < last) {
                    if (bw2 > 0.0f) {
                        xr[r] = sr + ((A0r * p2r) - (A0i * p2i) + (A1r * p1r) - (A1i * p1i));
                        xi[r] = si + ((A0i * p2r) + (A0r * p2i) + (A1i * p1r) + (A1r * p1i));
                    } else {
                        xr[r] = sr;
                        xi[r] = si;
                    }
                }
                p1r = p2r;
                p1i = p2i;
                p2r = sr;
                p2i = si;
                __builtin_amdgcn_sched_barrier(0);
            }
        }

        // ---------- HF adjustment (A/sbr/HFAdjustment.java) ----------
        const int m = u - kx;
        const bool band = m >= 0 && m < M;
        // estimate_current_envelope (:82-138)
        if (R.flags & kSbrInterpol) {
            float acc[5] = {0, 0, 0, 0, 0};
#pragma unroll
            for (int r = 2; r < 40; r++) {
                const float en = (xr[r] * xr[r]) + (xi[r] * xi[r]);
                const int i = r - 2;
#pragma unroll
                for (int l = 0; l < 5; l++)
                    if (l < L_E && i >= R.t_E[l] && i < R.t_E[l + 1]) acc[l] += en;
            }
#pragma unroll
            for (int l = 0; l < 5; l++) {
                if (l < L_E && band) {
                    float div = (float)(R.t_E[l + 1] - R.t_E[l]);
                    if (div == 0.0f) div = 1.0f;
                    L.ecurr[l][m] = __fdiv_rn(acc[l], div);
                }
            }
        } else {
            // band-group averages: nrg over rows (outer) and bands of the group (inner)
            for (int l = 0; l < L_E; l++) {
                const int fl = R.f[l];
                const int nb = fl ? T.n_hi : T.n_lo;
                int k_l = -1, k_h = -1;
                for (int p = 0; p < nb; p++)
                    if (u >= T.f_res[fl][p] && u < T.f_res[fl][p + 1]) {
                        k_l = T.f_res[fl][p];
                        k_h = T.f_res[fl][p + 1];
                    }
                int maxw = 0;
                for (int p = 0; p < nb; p++) maxw = max(maxw, (int)T.f_res[fl][p + 1] - (int)T.f_res[fl][p]);
                const int w = k_h - k_l;
                float nrg = 0.0f;
#pragma unroll
                for (int r = 2; r < 40; r++) {
                    const float en = (xr[r] * xr[r]) + (xi[r] * xi[r]);
                    const int i = r - 2;
                    if (i >= R.t_E[l] && i < R.t_E[l + 1]) {
                        for (int d = 0; d < maxw; d++) {
                            const float v = shfl(en, (u + d) & 63);
                            if (u == k_l && d < w) nrg += v;
                        }
                    }
                }
                int rows = R.t_E[l + 1] - R.t_E[l];
                float div = (float)(rows * w);
                if (div == 0.0f) div = 1.0f;
                const float own = __fdiv_rn(nrg, div);
                const float val = shfl(own, k_l >= 0 ? k_l : u);
                if (band && k_l >= 0) L.ecurr[l][m] = val;
            }
        }
        for (int i = u; i < 5 * 64; i += 64) {
            (&L.gl[0][0])[i] = 0.0f;
            (&L.ql[0][0])[i] = 0.0f;
            (&L.sl[0][0])[i] = 0.0f;
        }
        __syncthreads();

        // calculate_gain (:240-415).  Per envelope: (1) lanes m evaluate everything that does not
        // depend on the limiter (Q_M, S_M, the unlimited G) into LDS; (2) one lane per limiter
        // band walks its bands in order (acc1/acc2, G_max, limiting, den, G_boost) from LDS.
        {
            const int NL = T.N_L[s_lim];
            const float EPS = 1e-12f;
            int eo = (int)R.e_off;
            for (int l = 0; l < L_E; l++) {
                const int fl = R.f[l];
                const int tnb = R.tnb[l];
                const bool delta1 = !((R.no_noise >> l) & 1);
                const uint64_t smask = R.s_index[l], mmask = R.s_mapped[l];
                if (band) {
                    const int nb = T.noise_map[s_lim][m];
                    const float Qd = R.q_div[tnb][nb], Qd2 = R.q_div2[tnb][nb];
                    const float Eom = A.epool[eo + T.res_map[s_lim][fl][m]];
                    const float Ec = L.ecurr[l][m];
                    const bool sidx = (smask >> m) & 1, smap = (mmask >> m) & 1;
                    float G = __fdiv_rn(Eom, 1.0f + Ec);
                    if (!smap && delta1) G *= Qd;
                    else if (smap) G *= Qd2;
                    L.gq_eo[m] = Eom;
                    L.gq_qm[m] = Eom * Qd2;
                    L.gq_sm[m] = sidx ? Eom * Qd : 0.0f;
                    L.gq_g[m] = G;
                }
                eo += fl ? T.n_hi : T.n_lo;
                __syncthreads();
                for (int kb = u; kb < NL; kb += 64) {
                    const int ml1 = T.lim[s_lim][kb], ml2 = T.lim[s_lim][kb + 1];
                    float acc1 = 0.0f, acc2 = 0.0f;
                    for (int mm = ml1; mm < ml2; mm++) {
                        acc1 += L.gq_eo[mm];
                        acc2 += L.ecurr[l][mm];
                    }
                    float G_max = __fdiv_rn(EPS + acc1, EPS + acc2) * R.lim_gain;
                    G_max = java_minf(G_max, 1e10f);
                    float den = 0.0f;
                    for (int mm = ml1; mm < ml2; mm++) {
                        const bool sidx = (smask >> mm) & 1;
                        const float Q_M = L.gq_qm[mm], S_M = L.gq_sm[mm], G = L.gq_g[mm], Ec = L.ecurr[l][mm];
                        if (sidx) den += S_M;
                        float Ql, Gl;
                        if (G_max > G) {
                            Ql = Q_M;
                            Gl = G;
                        } else {
                            Ql = __fdiv_rn(Q_M * G_max, G);
                            Gl = G_max;
                        }
                        den += Ec * Gl;
                        if (!sidx && l != R.l_A) den += Ql;
                        L.gl[l][mm] = Gl;
                        L.ql[l][mm] = Ql;
                    }
                    float G_boost = __fdiv_rn(acc1 + EPS, den + EPS);
                    G_boost = java_minf(G_boost, 2.51188643f);
                    for (int mm = ml1; mm < ml2; mm++) {
                        L.gl[l][mm] = sqrtf(L.gl[l][mm] * G_boost);
                        L.ql[l][mm] = sqrtf(L.ql[l][mm] * G_boost);
                        const float sm = L.gq_sm[mm];
                        L.sl[l][mm] = sm != 0.0f ? sqrtf(sm * G_boost) : 0.0f;
                    }
                }
                __syncthreads();
            }
        }

        // hf_assembly (:140-238): lane k = m + kx
        {
            const int mi = band ? m : 0;
            const bool smooth = (R.flags & kSbrSmooth) != 0;
            if (R.flags & kSbrReset) {
                const float g0 = L.gl[0][mi], q0 = L.ql[0][mi];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    gr[j] = g0;
                    qr[j] = q0;
                }
                gidx = 4;
            }
            const float* noise = A.noise;
            const float rev = (u & 1) ? -1.0f : 1.0f;
#pragma unroll
            for (int r = 2; r < 40; r++) {
                const int i = r - 2;
                if (i < first || i >= last) continue;
                int l = 0;
                for (int j = 1; j < L_E; j++)
                    if (i >= R.t_E[j]) l = j;
                const bool no_noise = (R.no_noise >> l) & 1;
                const float gnew = L.gl[l][mi], qnew = L.ql[l][mi], S = L.sl[l][mi];
#pragma unroll
                for (int j = 0; j < 5; j++) {
                    if (j == gidx) {
                        gr[j] = gnew;
                        qr[j] = qnew;
                    }
                }
                float G_filt = 0.0f, Q_filt = 0.0f;
                if (smooth && !no_noise) {
                    int ri = gidx;
#pragma unroll
                    for (int n = 0; n <= 4; n++) {
                        const float h = n == 0 ? 0.03183050093751f : n == 1 ? 0.11516383427084f
                                      : n == 2 ? 0.21816949906249f : n == 3 ? 0.30150283239582f : 0.33333333333333f;
                        ri++;
                        if (ri >= 5) ri -= 5;
                        float gv = gr[0], qv = qr[0];
#pragma unroll
                        for (int j = 1; j < 5; j++)
                            if (j == ri) {
                                gv = gr[j];
                                qv = qr[j];
                            }
                        G_filt += gv * h;
                        Q_filt += qv * h;
                    }
                } else {
                    G_filt = gnew;
                    Q_filt = qnew;
                }
                Q_filt = (S != 0.0f || no_noise) ? 0.0f : Q_filt;
                const int fi = (int)((R.noise0 + (uint32_t)(i - first) * (uint32_t)M + (uint32_t)mi + 1u) & 511u);
                const int fs = (int)((R.sine0 + (uint32_t)(i - first)) & 3u);
                if (band) {
                    const float nr = noise[2 * fi], ni = noise[2 * fi + 1];
                    float vr = G_filt * xr[r] + (Q_filt * nr);
                    float vi = G_filt * xi[r] + (Q_filt * ni);
                    const float phr = fs == 0 ? 1.0f : fs == 2 ? -1.0f : 0.0f;
                    const float phi = fs == 1 ? 1.0f : fs == 3 ? -1.0f : 0.0f;
                    vr += S * phr;
                    vi += (rev * S) * phi;
                    xr[r] = vr;
                    xi[r] = vi;
                }
                gidx = gidx + 1 >= 5 ? 0 : gidx + 1;
                __builtin_amdgcn_sched_barrier(0);
            }
        }

        // ---------- synthesis (A/sbr/SynthesisFilterbank64.java:9-79) + PCM ----------
        const float scale = 1.f / 64.f;
        const int kcur = kx + M, kprev = R.kx_prev + R.M_prev;
#pragma unroll
        for (int l = 0; l < 32; l++) {
            const int klim = l < first ? kprev : kcur;
            const float Xr = u < klim ? xr[l + 2] : 0.0f;
            const float Xi = u < klim ? xi[l + 2] : 0.0f;
            // DCT inputs: d = 0: real parts (in_real1[e] = X[2e], in_imag1[e] = X[63-2e]);
            //             d = 1: imag parts (in_real2[e] = X[63-2e], in_imag2[e] = X[2e])
            const float ar = shfl(Xr, 2 * e), br = shfl(Xr, 63 - 2 * e);
            const float ai = shfl(Xi, 2 * e), bi = shfl(Xi, 63 - 2 * e);
            const float in_r = scale * (half ? bi : ar);
            const float in_i = scale * (half ? ai : br);
            float orr, oi;
            dct4(K, e, hb, in_r, in_i, orr, oi);
            // v block (:123-129): d=0 lanes write v[2n], v[127-2n]; d=1 lanes v[2n+1], v[126-2n]
            const float Ap = shfl(orr, u ^ 32);
            const float Bp = shfl(oi, 32 + (31 - e));
            const float Cp = shfl(oi, 31 - e);
            float* vb = L.vring[vpos];
            if (!half) {
                vb[2 * e] = Ap - orr;
                vb[127 - 2 * e] = Ap + orr;
            } else {
                vb[2 * e + 1] = Bp + Cp;
                vb[126 - 2 * e] = Bp - Cp;
            }
            __syncthreads();
            // window (:134-146)
            const float* v0 = L.vring[vpos];
            const float* v1 = L.vring[(vpos + 9) % 10];
            const float* v2 = L.vring[(vpos + 8) % 10];
            const float* v3 = L.vring[(vpos + 7) % 10];
            const float* v4 = L.vring[(vpos + 6) % 10];
            const float* v5 = L.vring[(vpos + 5) % 10];
            const float* v6 = L.vring[(vpos + 4) % 10];
            const float* v7 = L.vring[(vpos + 3) % 10];
            const float* v8 = L.vring[(vpos + 2) % 10];
            const float* v9 = L.vring[(vpos + 1) % 10];
            const float out = (v0[u] * cw[0]) + (v1[64 + u] * cw[1]) + (v2[u] * cw[2]) + (v3[64 + u] * cw[3]) +
                              (v4[u] * cw[4]) + (v5[64 + u] * cw[5]) + (v6[u] * cw[6]) + (v7[64 + u] * cw[7]) +
                              (v8[u] * cw[8]) + (v9[64 + u] * cw[9]);
            vpos = vpos == 9 ? 0 : vpos + 1;
            __syncthreads();  // window reads done before the next slot overwrites the oldest block
            if (emit) {
                const size_t n = (size_t)f * 2048 + 64 * l + u;
                if (A.out_mode & JAAD_PCM_FLOAT32) {
                    float* o = reinterpret_cast<float*>(A.pcm) + 2 * n;
                    if (nch == 2) o[c] = out;
                    else o[0] = o[1] = out;
                } else {
                    uint32_t s16 = (uint32_t)(uint16_t)(int16_t)java_round16(out);
                    if (!(A.out_mode & JAAD_PCM_LITTLE_ENDIAN)) s16 = ((s16 & 0xFF) << 8) | (s16 >> 8);
                    uint16_t* o = reinterpret_cast<uint16_t*>(A.pcm) + 2 * n;
                    if (nch == 2) o[c] = (uint16_t)s16;
                    else o[0] = o[1] = (uint16_t)s16;
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        carry_shift();
        __syncthreads();
    };

    const uint32_t f0 = ck.frame0;
    const bool prefix = (ck.flags & kSbrChunkPrefix) != 0;
    if (prefix) {
        // rows 0..7 of frame f0-1 = analysis slots 24..31 of frame f0-2 (their ring window lies
        // inside f0-2); frame f0-1 then runs in full without output (iteration j = -1)
        const size_t cf2 = (size_t)(f0 - 2) * nch + c;
        const int kx2 = A.tabs[A.recs[cf2].table].kx;
        load_window(nullptr, A.time + cf2 * 1024);
        analysis(12, kx2);
        carry_shift();
        __syncthreads();
    }
    for (int j = prefix ? -1 : 0; j < (int)ck.n; j++) {
        const int f = (int)f0 + j;
        const float* tail = (j == 0 && !prefix) ? tail_src : A.time + ((size_t)(f - 1) * nch + c) * 1024 + 736;
        process(f, tail, j >= 0);
    }
    if (ck.flags & kSbrChunkStore) {
        SbrChState& S = A.state_out[(size_t)ck.slot * 2 + c];
#pragma unroll
        for (int r = 0; r < 8; r++) {
            S.carry[r][u][0] = xr[r];
            S.carry[r][u][1] = xi[r];
        }
        // vhist[0..8] = oldest..newest = ring[(vpos + 1 + j) mod 10]
        for (int i = u; i < 9 * 128; i += 64) {
            const int j = i >> 7, o = i & 127;
            (&S.vhist[0][0])[i] = L.vring[(vpos + 1 + j) % 10][o];
        }
        const float* last = ck.n ? A.time + ((size_t)(f0 + ck.n - 1) * nch + c) * 1024 + 736 : tail_src;
        for (int i = u; i < 288; i += 64) S.tail[i] = last ? last[i] : 0.0f;
#pragma unroll
        for (int j = 0; j < 5; j++) {
            S.gq[0][j][u] = gr[j];
            S.gq[1][j][u] = qr[j];
        }
        if (u == 0) S.gq_index = (uint32_t)gidx;
    }
}

}  // namespace

hipError_t launch_sbr(const SbrArgs& a, hipStream_t stream)
{
    if (a.n_chunks == 0) return hipSuccess;
    hipLaunchKernelGGL(sbr_kernel, dim3(a.n_chunks), dim3(64), 0, stream, a);
    return hipGetLastError();
}

}  // namespace jaad

// ---------------------------------------------------------------------------------------------
// internal self-test entry points (not in the public header): the distributed DCT-IV on its own
// ---------------------------------------------------------------------------------------------
namespace jaad {
namespace {
__global__ void dct_test_kernel(const float* dct, const float* in_re, const float* in_im, float* out_re,
                                float* out_im, int n)
{
    const int u = lane_id();
    const int e = u & 31, hb = u & 32;
    const int v = blockIdx.x * 2 + (u >> 5);
    DctConst K;
    const float* wr = dct + 192;
    const float* wi = dct + 208;
    K.t0 = dct[e];
    K.t32 = dct[e + 32];
    K.t64 = dct[e + 64];
    K.t96 = dct[e + 96];
    K.t128 = dct[e + 128];
    K.t160 = dct[e + 160];
    K.w1r = wr[e & 15];
    K.w1i = wi[e & 15];
    K.w2r = wr[2 * (e & 7)];
    K.w2i = wi[2 * (e & 7)];
    K.w3 = (e & 3) == 1 ? wr[4] : wr[12];
    const int vv = v < n ? v : n - 1;
    float orr, oi;
    dct4(K, e, hb, in_re[32 * vv + e], in_im[32 * vv + e], orr, oi);
    if (v < n) {
        out_re[32 * v + e] = orr;
        out_im[32 * v + e] = oi;
    }
}
}  // namespace
}  // namespace jaad

extern "C" int jaad__sbr_dct_test(const float* dct_dev, const float* in_re, const float* in_im, float* out_re,
                                  float* out_im, int n)
{
    hipLaunchKernelGGL(jaad::dct_test_kernel, dim3((n + 1) / 2), dim3(64), 0, nullptr, dct_dev, in_re, in_im, out_re,
                       out_im, n);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -3;
}

namespace jaad {
namespace {
__global__ void math_test_kernel(const float* a, const float* b, float* sq, float* dv, int n)
{
    const int i = blockIdx.x * 64 + lane_id();
    if (i < n) {
        sq[i] = (float)__dsqrt_rn((double)a[i]);
        dv[i] = sqrtf(a[i]);
    }
}
}  // namespace
}  // namespace jaad

extern "C" int jaad__math_test(const float* a, const float* b, float* sq, float* dv, int n)
{
    hipLaunchKernelGGL(jaad::math_test_kernel, dim3((n + 63) / 64), dim3(64), 0, nullptr, a, b, sq, dv, n);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -3;
}
