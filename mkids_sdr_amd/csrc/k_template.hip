// MakeTemplate (DataReadout/ReadoutControls/lib/pulses.py:239-427) and the
// near-optimal filter it stubs (pulses.py:398; PulseAnalysis.coeff, pulses.py:59), on device.
//
// The reference loops over one resonator's pulses (I, Q float32 [P][2000]) twice in Python; here
// every pulse is one 256-thread workgroup:
//   prep     I += I1m - median(I[1:900]) (in place: the reference edits its table, so the first
//            1000 pulses are re-referenced again in pass 2), P1 = atan2(Q, I) (float32), numpy
//            unwrap (float32, sequential cumsum), rad2deg, linear polyfit over [0:900]+[1800:]
//            (float64), P3 = P2 - fit, bad = |mean(P3[:100]) - mean(P3[1900:])| > 2 std(P3[:100])
//   pass 1   peak = max P3[980:1050]; 15..120 deg; ploc (first index == peak) in 980..1020;
//            row = roll(P3, 1000 - ploc) / max
//   pass 2   ploc = argmax(convolve(tP[900:1500], P3)) - 1160, peak = P3[1000 + ploc] within
//            pm +- 4 pdev, |ploc| <= 30; row = roll(P3, -ploc) / max; noise row =
//            |DFT800(deg2rad(row-before-normalisation[50:850]))|^2
// Accumulations over pulses run column-parallel in pulse order (the reference's += order), the
// medians are exact order statistics (workgroup radix select), pm / pdev / std / mean follow
// numpy's pairwise float64 summation. Results agree with oracle/template_ref.py to float rounding
// (atan2f and the least-squares fit differ in the last bits), and every accept/skip decision away
// from a threshold is identical (tests/test_template.py).
#include "mkid_internal.h"

namespace mkid {

constexpr int kTN = 2000;   // samples per pulse (RawPulse.I, pulses.py:42)
constexpr int kTNoise = 800;
constexpr int kTB = 256;

__device__ __forceinline__ uint32_t fkey(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fval(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// k-th smallest (0-based) of get(0..n-1), exact, by the whole workgroup (4 radix-8 passes)
template <typename G>
__device__ float wg_select(G get, int n, int k) {
    __shared__ uint32_t hist[256];
    __shared__ uint32_t s_prefix, s_k;
    uint32_t prefix = 0, mask = 0;
    if (threadIdx.x == 0) s_k = (uint32_t)k;
    for (int shift = 24; shift >= 0; shift -= 8) {
        for (int b = threadIdx.x; b < 256; b += blockDim.x) hist[b] = 0;
        __syncthreads();
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            const uint32_t key = fkey(get(i));
            if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t kk = s_k, cum = 0, sel = 255;
            for (int b = 0; b < 256; ++b) {
                if (cum + hist[b] > kk) { sel = (uint32_t)b; break; }
                cum += hist[b];
            }
            s_k = kk - cum;
            s_prefix = prefix | (sel << shift);
        }
        __syncthreads();
        prefix = s_prefix;
        mask |= 255u << shift;
        __syncthreads();
    }
    return fval(prefix);
}

// np.median of float32 data: middle element, or the float32 mean of the two middle elements
template <typename G>
__device__ float wg_median(G get, int n) {
    if (n & 1) return wg_select(get, n, n / 2);
    const float a = wg_select(get, n, n / 2 - 1);
    const float b = wg_select(get, n, n / 2);
    return (a + b) / 2.0f;
}

// numpy pairwise_sum over a double array (loops_utils.h.src), n <= 128 leaf / halving
__device__ double pw_leaf_d(const double* a, int n) {
    if (n < 8) {
        double r = 0.0;
        for (int i = 0; i < n; ++i) r += a[i];
        return r;
    }
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
}
__device__ double pw_sum_d(const double* a, int n) {
    if (n <= 128) return pw_leaf_d(a, n);
    // recursion n -> (n2 = n/2 - (n/2)%8, n - n2), unrolled with an explicit stack
    struct Fr { int o, n, state; double left; };
    Fr st[20];
    int sp = 0;
    st[0] = Fr{0, n, 0, 0.0};
    double ret = 0.0;
    while (sp >= 0) {
        Fr& f = st[sp];
        if (f.n <= 128) { ret = pw_leaf_d(a + f.o, f.n); --sp; continue; }
        int n2 = f.n / 2;
        n2 -= n2 % 8;
        if (f.state == 0) { f.state = 1; st[sp + 1] = Fr{f.o, n2, 0, 0.0}; ++sp; }
        else if (f.state == 1) { f.left = ret; f.state = 2; st[sp + 1] = Fr{f.o + n2, f.n - n2, 0, 0.0}; ++sp; }
        else { ret = f.left + ret; --sp; }
    }
    return ret;
}
__device__ double np_mean(const double* a, int n) { return pw_sum_d(a, n) / (double)n; }
// np.std: sqrt(mean(abs(x - mean(x))**2)); tmp is scratch of n doubles
__device__ double np_std(const double* a, int n, double* tmp) {
    const double m = np_mean(a, n);
    for (int i = 0; i < n; ++i) {
        const double d = fabs(a[i] - m);
        tmp[i] = d * d;
    }
    return sqrt(pw_sum_d(tmp, n) / (double)n);
}

// numpy float mod (npy_divmodf): sign of the divisor
__device__ __forceinline__ float np_modf(float a, float b) {
    float m = fmodf(a, b);
    if (m != 0.0f) {
        if ((b < 0.0f) != (m < 0.0f)) m += b;
    } else {
        m = copysignf(0.0f, b);
    }
    return m;
}

struct TplArgs {
    float* I;            // [P][2000] work copy, re-referenced in place
    float* Q;
    int64_t P;
    float I1m, Q1m;
    const double* tP;    // pass-1 template (pass 2)
    double pm, pdev;     // pass-1 peak statistics (pass 2)
    double* rows;        // [P][2000] normalised aligned pulses
    double* nrows;       // [P][800] noise periodograms (pass 2)
    int32_t* accept;     // [P]
    double* peaks;       // [P] pass-1 peak (appended iff not bad)
    int32_t* appended;   // [P]
    int pass;
};

// One pulse: prep (re-reference, phase, unwrap, baseline) then the pass's selection.
__global__ __launch_bounds__(kTB) void k_tpl_pulse(TplArgs a) {
    const int64_t j = blockIdx.x;
    if (j >= a.P) return;
    __shared__ float sI[kTN], sQ[kTN], sP2[kTN];
    __shared__ double sP3[kTN];
    __shared__ double sA[600];
    __shared__ double red[kTB];
    __shared__ int redi[kTB];
    __shared__ double s_fit[2];
    __shared__ int s_bad;
    float* gI = a.I + j * kTN;
    float* gQ = a.Q + j * kTN;
    const int t0 = threadIdx.x;
    for (int t = t0; t < kTN; t += kTB) { sI[t] = gI[t]; sQ[t] = gQ[t]; }
    __syncthreads();
    // I += I1m - median(I[1:900]) (float32), written back: the reference edits its table
    const float mI = wg_median([&](int i) { return sI[1 + i]; }, 899);
    const float mQ = wg_median([&](int i) { return sQ[1 + i]; }, 899);
    const float dI = a.I1m - mI, dQ = a.Q1m - mQ;
    for (int t = t0; t < kTN; t += kTB) {
        sI[t] += dI;
        sQ[t] += dQ;
        gI[t] = sI[t];
        gQ[t] = sQ[t];
        sP2[t] = atan2f(sQ[t] - 0.0f, sI[t] - 0.0f);  // P1 (xc = yc = 0, pulses.py:274-275)
    }
    __syncthreads();
    // np.unwrap (float32: period 2pi, discont pi) + rad2deg, sequential like the reference's cumsum
    if (t0 == 0) {
        const float hi = 3.14159265358979311600f, per = 6.28318530717958623200f;
        const float r2d = 180.0f / 3.14159265358979311600f;  // numpy float32 rad2deg: 180.0f/NPY_PIf
        float cum = 0.0f, prev = sP2[0];
        sP2[0] = sP2[0] * r2d;
        for (int t = 1; t < kTN; ++t) {
            const float p = sP2[t];
            const float dd = p - prev;
            float ddmod = np_modf(dd - (-hi), per) + (-hi);
            if (ddmod == -hi && dd > 0.0f) ddmod = hi;
            float corr = ddmod - dd;
            if (fabsf(dd) < hi) corr = 0.0f;
            cum += corr;
            prev = p;
            sP2[t] = (p + cum) * r2d;
        }
    }
    __syncthreads();
    // linear least squares of P2 on x = 2t over t in [0,900) u [1800,2000)  (polyfit deg 1)
    {
        double sx = 0, sy = 0;
        for (int t = t0; t < kTN; t += kTB)
            if (t < 900 || t >= 1800) { sx += 2.0 * t; sy += (double)sP2[t]; }
        red[t0] = sx;
        __syncthreads();
        for (int o = kTB / 2; o > 0; o >>= 1) { if (t0 < o) red[t0] += red[t0 + o]; __syncthreads(); }
        const double xm = red[0] / 1100.0;
        __syncthreads();
        red[t0] = sy;
        __syncthreads();
        for (int o = kTB / 2; o > 0; o >>= 1) { if (t0 < o) red[t0] += red[t0 + o]; __syncthreads(); }
        const double ym = red[0] / 1100.0;
        __syncthreads();
        double sxy = 0, sxx = 0;
        for (int t = t0; t < kTN; t += kTB)
            if (t < 900 || t >= 1800) {
                const double dx = 2.0 * t - xm;
                sxy += dx * ((double)sP2[t] - ym);
                sxx += dx * dx;
            }
        red[t0] = sxy;
        __syncthreads();
        for (int o = kTB / 2; o > 0; o >>= 1) { if (t0 < o) red[t0] += red[t0 + o]; __syncthreads(); }
        const double cxy = red[0];
        __syncthreads();
        red[t0] = sxx;
        __syncthreads();
        for (int o = kTB / 2; o > 0; o >>= 1) { if (t0 < o) red[t0] += red[t0 + o]; __syncthreads(); }
        if (t0 == 0) {
            s_fit[0] = cxy / red[0];
            s_fit[1] = ym - s_fit[0] * xm;
        }
        __syncthreads();
    }
    for (int t = t0; t < kTN; t += kTB) sP3[t] = (double)sP2[t] - (s_fit[0] * (2.0 * t) + s_fit[1]);
    __syncthreads();
    if (t0 == 0) {
        double* tmp = sA;  // scratch (100 doubles)
        const double sd = np_std(sP3, 100, tmp);
        s_bad = fabs(np_mean(sP3, 100) - np_mean(sP3 + 1900, 100)) > sd * 2.0;
    }
    __syncthreads();
    if (s_bad) {
        if (t0 == 0) {
            a.accept[j] = 0;
            if (a.pass == 1) a.appended[j] = 0;
        }
        return;
    }
    // max over all of P3 (normalisation) and the pass's peak search
    double mx = -INFINITY;
    for (int t = t0; t < kTN; t += kTB) mx = fmax(mx, sP3[t]);
    red[t0] = mx;
    __syncthreads();
    for (int o = kTB / 2; o > 0; o >>= 1) { if (t0 < o) red[t0] = fmax(red[t0], red[t0 + o]); __syncthreads(); }
    const double pmax = red[0];
    __syncthreads();
    int shift = 0;
    bool ok = true;
    if (a.pass == 1) {
        double pk = -INFINITY;
        for (int t = 980 + t0; t < 1050; t += kTB) pk = fmax(pk, sP3[t]);
        red[t0] = pk;
        __syncthreads();
        for (int o = kTB / 2; o > 0; o >>= 1) { if (t0 < o) red[t0] = fmax(red[t0], red[t0 + o]); __syncthreads(); }
        const double peak = red[0];
        __syncthreads();
        int first = kTN;
        for (int t = t0; t < kTN; t += kTB)
            if (sP3[t] == peak && t < first) first = t;
        redi[t0] = first;
        __syncthreads();
        for (int o = kTB / 2; o > 0; o >>= 1) { if (t0 < o) redi[t0] = min(redi[t0], redi[t0 + o]); __syncthreads(); }
        const int ploc = redi[0];
        if (t0 == 0) { a.peaks[j] = peak; a.appended[j] = 1; }
        ok = !(peak < 15.0 || peak > 120.0) && !(ploc < 980 || ploc > 1020);
        shift = 1000 - ploc;
    } else {
        // conv[n] = sum_k tP[900+k] P3[n-k], n in [0, 2599); first argmax
        for (int k = t0; k < 600; k += kTB) sA[k] = a.tP[900 + k];
        __syncthreads();
        double best = -INFINITY;
        int bi = 1 << 30;
        for (int n = t0; n < 2599; n += kTB) {
            const int klo = n - (kTN - 1) > 0 ? n - (kTN - 1) : 0, khi = n < 599 ? n : 599;
            double s = 0.0;
            for (int k = klo; k <= khi; ++k) s += sA[k] * sP3[n - k];
            if (s > best) { best = s; bi = n; }
        }
        red[t0] = best;
        redi[t0] = bi;
        __syncthreads();
        for (int o = kTB / 2; o > 0; o >>= 1) {
            if (t0 < o && (red[t0 + o] > red[t0] || (red[t0 + o] == red[t0] && redi[t0 + o] < redi[t0]))) {
                red[t0] = red[t0 + o];
                redi[t0] = redi[t0 + o];
            }
            __syncthreads();
        }
        const int ploc = redi[0] - 1160;
        int pi = 1000 + ploc;
        if (pi < 0) pi += kTN;  // numpy negative index
        const bool inr = pi >= 0 && pi < kTN;  // out of range: the reference raises; skipped here
        const double peak = inr ? sP3[pi] : 0.0;
        ok = inr && !(peak < a.pm - 4.0 * a.pdev || peak > a.pm + 4.0 * a.pdev) && !(ploc < -30 || ploc > 30);
        shift = -ploc;
    }
    if (t0 == 0) a.accept[j] = ok ? 1 : 0;
    if (!ok) return;
    // row = roll(P3, shift) / max(P3)
    double* row = a.rows + j * kTN;
    for (int t = t0; t < kTN; t += kTB) {
        int src = t - shift;
        src %= kTN;
        if (src < 0) src += kTN;
        row[t] = sP3[src] / pmax;
    }
    if (a.pass == 2) {
        // |DFT800(deg2rad(roll(P3)[50:850]))|^2, direct in float64 with a twiddle table in the
        // (now free) sI/sQ space
        __syncthreads();
        __shared__ double win[kTNoise];
        double* twr = reinterpret_cast<double*>(sI);  // 800 doubles = 6400 B <= 8000 B
        double* twi = reinterpret_cast<double*>(sQ);
        for (int k = t0; k < kTNoise; k += kTB) {
            double sn, cs;
            sincospi(-2.0 * k / kTNoise, &sn, &cs);
            twr[k] = cs;
            twi[k] = sn;
        }
        for (int t = t0; t < kTNoise; t += kTB) {
            int src = 50 + t - shift;
            src %= kTN;
            if (src < 0) src += kTN;
            win[t] = sP3[src] * 0.017453292519943295;
        }
        __syncthreads();
        double* nrow = a.nrows + j * kTNoise;
        for (int f = t0; f < kTNoise; f += kTB) {
            double re = 0.0, im = 0.0;
            int ph = 0;
            for (int n = 0; n < kTNoise; ++n) {
                re += win[n] * twr[ph];
                im += win[n] * twi[ph];
                ph += f;
                if (ph >= kTNoise) ph -= kTNoise;
            }
            nrow[f] = re * re + im * im;
        }
    }
}

// column sums over accepted rows in pulse order; out[t] = sum / count
__global__ void k_tpl_colsum(const double* rows, const int32_t* accept, int64_t P, int width, double* out,
                             double* count) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= width) return;
    double s = 0.0, n = 0.0;
    for (int64_t j = 0; j < P; ++j)
        if (accept[j]) { s += rows[j * width + t]; n += 1.0; }
    out[t] = s / n;
    if (t == 0) *count = n;
}

// global reference medians I1m, Q1m over pulses [0, min(P,100)) x samples [0, 900)
__global__ void k_tpl_refmed(const float* I, const float* Q, int64_t P, float* out) {
    const int np = (int)(P < 100 ? P : 100);
    const int n = np * 900;
    const float mi = wg_median([&](int i) { return I[(int64_t)(i / 900) * kTN + i % 900]; }, n);
    const float mq = wg_median([&](int i) { return Q[(int64_t)(i / 900) * kTN + i % 900]; }, n);
    if (threadIdx.x == 0) { out[0] = mi; out[1] = mq; }
}

// pm, pdev: median / std of appended pass-1 peaks > 15 (pulses.py:334-336), in pulse order
__global__ void k_tpl_peakstats(const double* peaks, const int32_t* appended, int64_t P, double* out,
                                double* scratch) {
    if (threadIdx.x != 0) return;
    int n = 0;
    for (int64_t j = 0; j < P; ++j)
        if (appended[j] && peaks[j] > 15.0) scratch[n++] = peaks[j];
    out[2] = n;
    if (n == 0) { out[0] = out[1] = NAN; return; }
    // std in pulse order (pairwise), then the median on a sorted copy (insertion sort, n <= 1000)
    double* tmp = scratch + P;
    out[1] = np_std(scratch, n, tmp);
    for (int i = 1; i < n; ++i) {
        const double v = scratch[i];
        int k = i - 1;
        while (k >= 0 && scratch[k] > v) { scratch[k + 1] = scratch[k]; --k; }
        scratch[k + 1] = v;
    }
    out[0] = (n & 1) ? scratch[n / 2] : (scratch[n / 2 - 1] + scratch[n / 2]) / 2.0;
}

// near-optimal filter: s = deg2rad(template[pk-pre : pk-pre+800]); H = S / J, H[0] = 0;
// g = real(ifft(H)) (correlation weights), g /= g.s; coeff = g[pre-10 : pre-10+ncoeff]
__global__ void k_tpl_optfilt(const double* tpl, const double* noise, int pre, int ncoeff, double* coeff,
                              double* work) {
    __shared__ double s[kTNoise];
    __shared__ double red[kTB];
    __shared__ int redi[kTB];
    const int t0 = threadIdx.x;
    double best = -INFINITY;
    int bi = kTN;
    for (int t = t0; t < kTN; t += kTB)
        if (tpl[t] > best || (tpl[t] == best && t < bi)) { best = tpl[t]; bi = t; }
    red[t0] = best;
    redi[t0] = bi;
    __syncthreads();
    for (int o = kTB / 2; o > 0; o >>= 1) {
        if (t0 < o && (red[t0 + o] > red[t0] || (red[t0 + o] == red[t0] && redi[t0 + o] < redi[t0]))) {
            red[t0] = red[t0 + o];
            redi[t0] = redi[t0 + o];
        }
        __syncthreads();
    }
    const int p0 = redi[0] - pre;
    for (int t = t0; t < kTNoise; t += kTB) {
        const int i = p0 + t;
        s[t] = (i >= 0 && i < kTN) ? tpl[i] * 0.017453292519943295 : 0.0;
    }
    __syncthreads();
    double* Hr = work;
    double* Hi = work + kTNoise;
    double* g = work + 2 * kTNoise;
    __shared__ double twr[kTNoise], twi[kTNoise];
    for (int k = t0; k < kTNoise; k += kTB) {
        double sn, cs;
        sincospi(-2.0 * k / kTNoise, &sn, &cs);
        twr[k] = cs;
        twi[k] = sn;
    }
    __syncthreads();
    for (int f = t0; f < kTNoise; f += kTB) {
        double re = 0.0, im = 0.0;
        int ph = 0;
        for (int n = 0; n < kTNoise; ++n) {
            re += s[n] * twr[ph];
            im += s[n] * twi[ph];
            ph += f;
            if (ph >= kTNoise) ph -= kTNoise;
        }
        const double J = noise[f];
        Hr[f] = f == 0 ? 0.0 : re / J;
        Hi[f] = f == 0 ? 0.0 : im / J;
    }
    __syncthreads();
    for (int m = t0; m < kTNoise; m += kTB) {
        double re = 0.0;
        int ph = 0;
        for (int f = 0; f < kTNoise; ++f) {
            re += Hr[f] * twr[ph] + Hi[f] * twi[ph];  // exp(+i theta) = conj(tw)
            ph += m;
            if (ph >= kTNoise) ph -= kTNoise;
        }
        g[m] = re / kTNoise;
    }
    __syncthreads();
    double d = 0.0;
    for (int m = t0; m < kTNoise; m += kTB) d += g[m] * s[m];
    red[t0] = d;
    __syncthreads();
    for (int o = kTB / 2; o > 0; o >>= 1) { if (t0 < o) red[t0] += red[t0 + o]; __syncthreads(); }
    const double norm = red[0];
    const int k0 = pre - 10;
    for (int i = t0; i < ncoeff; i += kTB) {
        const int m = k0 + i;
        coeff[i] = (m >= 0 && m < kTNoise) ? g[m] / norm : 0.0;
    }
}

hipError_t launch_make_template(float* I, float* Q, int64_t P, double* rows, double* nrows, int32_t* accept,
                                double* peaks, int32_t* appended, double* scratch, double* tP, double* tPf,
                                double* noise, double* stats, float* refmed, hipStream_t s) {
    // stats: [pm, pdev, npk, count1, count2]
    hipLaunchKernelGGL(k_tpl_refmed, dim3(1), dim3(1024), 0, s, I, Q, P, refmed);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    float rm[2];
    if ((e = hipMemcpyAsync(rm, refmed, 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    TplArgs a{I, Q, P < 1000 ? P : 1000, rm[0], rm[1], nullptr, 0, 0, rows, nrows, accept, peaks, appended, 1};
    hipLaunchKernelGGL(k_tpl_pulse, dim3((unsigned)a.P), dim3(kTB), 0, s, a);
    hipLaunchKernelGGL(k_tpl_colsum, dim3((kTN + 255) / 256), dim3(256), 0, s, rows, accept, a.P, kTN, tP,
                       stats + 3);
    hipLaunchKernelGGL(k_tpl_peakstats, dim3(1), dim3(64), 0, s, peaks, appended, a.P, stats, scratch);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    double st[4];
    if ((e = hipMemcpyAsync(st, stats, 32, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    if (!(st[3] > 0)) return hipErrorInvalidValue;  // no pulse passed the first pass
    TplArgs b = a;
    b.P = P;
    b.tP = tP;
    b.pm = st[0];
    b.pdev = st[1];
    b.pass = 2;
    hipLaunchKernelGGL(k_tpl_pulse, dim3((unsigned)P), dim3(kTB), 0, s, b);
    hipLaunchKernelGGL(k_tpl_colsum, dim3((kTN + 255) / 256), dim3(256), 0, s, rows, accept, P, kTN, tPf,
                       stats + 4);
    hipLaunchKernelGGL(k_tpl_colsum, dim3((kTNoise + 255) / 256), dim3(256), 0, s, nrows, accept, P, kTNoise,
                       noise, stats + 4);
    return hipGetLastError();
}

hipError_t launch_optimal_filter(const double* tpl, const double* noise, int pre, int ncoeff, double* coeff,
                                 double* work, hipStream_t s) {
    hipLaunchKernelGGL(k_tpl_optfilt, dim3(1), dim3(kTB), 0, s, tpl, noise, pre, ncoeff, coeff, work);
    return hipGetLastError();
}

}  // namespace mkid
