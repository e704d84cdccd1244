// Host-replay triggers of the reference, run on the device over Fix16_13 phase (SURVEY.md §8 a12,
// a13). The reference reads a phase snapshot and walks it in a Python while-loop:
//   rolling  pulse_triggering_v2.py:104-174 (same loop pulse_triggering_IQ.py:159-200):
//            bob = 100 + m; while bob < n: if bob + L > n: break;
//            if |mean(x[bob-m:bob]) - x[bob]| > T: hit, bob += L  else bob += 1
//   block    pulse_triggering.py:109-208, ROACH_Pulses.py:614-727: x[x < 0] += 360 (first form);
//            means over fixed blocks of A; the same walk with mean[bob // A], need / skip params.
// with x = raw * 360. / 2**16 * 4 / pi (pulse_triggering_v2.py:93-95), all in float64.
//
// Device form: (1) every candidate test |mean - x[j]| > T is independent of the walk, so one
// pass sets a bit per (channel, j); (2) one thread per channel walks its bit row, jumping to the
// next set bit with ffs. Means use numpy's pairwise summation order exactly (np.add.reduce on a
// contiguous float64 row: 8 accumulators up to 128 elements, halving above), so every
// comparison - and therefore every hit - matches the reference's numpy arithmetic bit for bit.
#include "mkid_internal.h"

namespace mkid {

__device__ __forceinline__ double raw_deg(int16_t r) {
    return (double)r * 360.0 / 65536.0 * 4.0 / 3.14159265358979311600;  // np.pi, left to right
}

struct RawRow {  // channel c of a [n][ld] int16 buffer, optionally wrapped to [0, 360)
    const int16_t* p;
    int64_t ld;
    int wrap;
    __device__ __forceinline__ double operator[](int64_t j) const {
        const double x = raw_deg(p[j * ld]);
        return (wrap && x < 0.0) ? x + 360.0 : x;
    }
};

// numpy pairwise_sum for n <= 128 (loops_utils.h.src): sequential below 8, else 8 accumulators
__device__ double pw_leaf(const RawRow& x, int64_t o, int64_t n) {
    if (n < 8) {
        double res = 0.0;
        for (int64_t i = 0; i < n; ++i) res += x[o + i];
        return res;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = x[o + j];
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += x[o + i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += x[o + i];
    return res;
}

// full pairwise_sum: recursion n -> (n2 = n/2 - (n/2)%8, n - n2) unrolled with an explicit stack
__device__ double pw_sum(const RawRow& x, int64_t o, int64_t n) {
    if (n <= 128) return pw_leaf(x, o, n);
    struct Fr { int64_t o, n; double left; int state; };
    Fr st[24];
    int sp = 0;
    st[0] = Fr{o, n, 0.0, 0};
    double ret = 0.0;
    while (sp >= 0) {
        Fr& f = st[sp];
        if (f.n <= 128) {
            ret = pw_leaf(x, f.o, f.n);
            --sp;
            continue;
        }
        int64_t n2 = f.n / 2;
        n2 -= n2 % 8;
        if (f.state == 0) {  // descend left
            f.state = 1;
            st[sp + 1] = Fr{f.o, n2, 0.0, 0};
            ++sp;
        } else if (f.state == 1) {  // left done -> descend right
            f.left = ret;
            f.state = 2;
            st[sp + 1] = Fr{f.o + n2, f.n - n2, 0.0, 0};
            ++sp;
        } else {  // both done
            ret = f.left + ret;
            --sp;
        }
    }
    return ret;
}

// rolling mode: bit j of row c set iff j >= m and |mean(x[j-m:j]) - x[j]| > thr
__global__ void k_replay_flags_rolling(const int16_t* raw, int64_t n, int64_t ld, int32_t nch, int32_t m,
                                       double thr, int32_t wrap, uint32_t* flags, int64_t nw) {
    const int c = blockIdx.y * blockDim.x + threadIdx.x;  // lanes = channels (coalesced rows)
    const int64_t w = blockIdx.x;
    if (c >= nch || w >= nw) return;
    const RawRow x{raw + c, ld, wrap};
    uint32_t bits = 0;
    for (int b = 0; b < 32; ++b) {
        const int64_t j = w * 32 + b;
        if (j >= n) break;
        if (j < m) continue;
        const double mean = pw_sum(x, j - m, m) / (double)m;
        if (fabs(mean - x[j]) > thr) bits |= 1u << b;
    }
    flags[(int64_t)c * nw + w] = bits;
}

__global__ void k_replay_block_means(const int16_t* raw, int64_t ld, int32_t nch, int32_t A, int64_t nmeans,
                                     int32_t wrap, double* means) {
    const int c = blockIdx.y * blockDim.x + threadIdx.x;
    const int64_t b = blockIdx.x;
    if (c >= nch || b >= nmeans) return;
    const RawRow x{raw + c, ld, wrap};
    means[(int64_t)c * nmeans + b] = pw_sum(x, b * A, A) / (double)A;
}

// block mode: bit j set iff j // A < nmeans and |mean[j // A] - x[j]| > thr
__global__ void k_replay_flags_block(const int16_t* raw, int64_t n, int64_t ld, int32_t nch, int32_t A,
                                     int64_t nmeans, double thr, int32_t wrap, const double* means,
                                     uint32_t* flags, int64_t nw) {
    const int c = blockIdx.y * blockDim.x + threadIdx.x;
    const int64_t w = blockIdx.x;
    if (c >= nch || w >= nw) return;
    const RawRow x{raw + c, ld, wrap};
    uint32_t bits = 0;
    for (int b = 0; b < 32; ++b) {
        const int64_t j = w * 32 + b;
        if (j >= n) break;
        const int64_t which = j / A;
        if (which >= nmeans) continue;
        if (fabs(means[(int64_t)c * nmeans + which] - x[j]) > thr) bits |= 1u << b;
    }
    flags[(int64_t)c * nw + w] = bits;
}

// the reference's while-loop, one thread per channel, jumping between candidate bits
__global__ void k_replay_walk(const uint32_t* flags, int64_t n, int64_t nw, int32_t nch, int64_t start,
                              int64_t need, int64_t skip, int64_t A, int64_t nmeans, int32_t* hits,
                              int32_t cap, int32_t* counts) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nch) return;
    const uint32_t* row = flags + (int64_t)c * nw;
    int32_t nh = 0;
    int64_t bob = start;
    while (bob < n) {
        // next candidate >= bob
        int64_t w = bob >> 5;
        uint32_t bits = w < nw ? row[w] & (~0u << (bob & 31)) : 0;
        while (bits == 0 && ++w < nw) bits = row[w];
        if (bits == 0) break;
        const int64_t f = w * 32 + __ffs(bits) - 1;
        // every index between bob and f failed the test; the loop's own exits come first
        if (f + need > n) break;                   // "if bob + need > n: break"
        if (A > 0 && f / A >= nmeans) break;       // mean[bob // A] out of range (reference: IndexError)
        if (nh < cap) hits[(int64_t)c * cap + nh] = (int32_t)f;
        ++nh;
        bob = f + skip;
    }
    counts[c] = nh;
}

hipError_t launch_replay(const int16_t* raw, int64_t n, int64_t ld, int32_t nch, int32_t mode, int32_t length,
                         int64_t start, int64_t need, int64_t skip, int32_t wrap, double thr, uint32_t* flags,
                         double* means, int32_t* hits, int32_t cap, int32_t* counts, hipStream_t s) {
    const int64_t nw = (n + 31) / 32;
    const int TB = 64;
    const unsigned gy = (unsigned)((nch + TB - 1) / TB);
    int64_t A = 0, nmeans = 0;
    if (mode == 0) {
        hipLaunchKernelGGL(k_replay_flags_rolling, dim3((unsigned)nw, gy), dim3(TB), 0, s, raw, n, ld, nch,
                           length, thr, wrap, flags, nw);
    } else {
        A = length;
        nmeans = n / A;
        if (nmeans > 0)
            hipLaunchKernelGGL(k_replay_block_means, dim3((unsigned)nmeans, gy), dim3(TB), 0, s, raw, ld, nch,
                               length, nmeans, wrap, means);
        hipLaunchKernelGGL(k_replay_flags_block, dim3((unsigned)nw, gy), dim3(TB), 0, s, raw, n, ld, nch,
                           length, nmeans, thr, wrap, means, flags, nw);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_replay_walk, dim3((unsigned)((nch + 255) / 256)), dim3(256), 0, s, flags, n, nw, nch,
                       start, need, skip, A, nmeans, hits, cap, counts);
    return hipGetLastError();
}

}  // namespace mkid
