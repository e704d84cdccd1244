// Packet compaction (exclusive scan over (channel, segment) counts) and stream-history rolls.
#include "mkid_internal.h"

namespace mkid {

// ---- compaction: exclusive scan of (channel, segment) packet counts, then copy -------------
// Three launches, all coalesced: (1) per-tile sums of TILE consecutive entries, (2) one block
// scans the tile sums (and writes the call's totals), (3) per tile: block-local exclusive scan +
// tile offset, each thread copies the packets of its entries; the same launch carries the call's
// history rolls as extra blocks (round 6: one launch fewer per call). Round 6 also: one entry per
// thread (with 8 the copy ran eight dependent load -> store chains in a row per thread:
// k_gather_events 16.7 -> 8.2 us per step at config 3, 13.3 -> 5.3 us at config 2); the block
// scans are wave scans plus one exchange of wave totals (k_tile_scan 7.8 -> 4.8 us); the tile scan
// folded into (1) as a last-block pass was slower (1024 blocks serialise on the done counter:
// k_tile_sums 4.9 -> 27 us).
constexpr int kCmpThreads = 256;
constexpr int kCmpEpt = 1;                       // entries per thread
constexpr int kCmpTile = kCmpThreads * kCmpEpt;  // entries per tile
constexpr int kScanThreads = 1024;

__device__ __forceinline__ void load_counts(const int32_t* counts, int64_t n_ent, int64_t e0,
                                            int32_t capseg, int (&v)[kCmpEpt], int64_t& raw,
                                            int64_t& kept) {
    raw = 0;
    kept = 0;
#pragma unroll
    for (int i = 0; i < kCmpEpt; ++i) {
        const int x = e0 + i < n_ent ? counts[e0 + i] : 0;
        raw += x;
        v[i] = x < capseg ? x : capseg;
        kept += v[i];
    }
}

// inclusive scan over the 64 lanes of a wave (6 shuffle steps, no barrier)
__device__ __forceinline__ int64_t wave_incl_scan(int64_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t y = __shfl_up(x, off, 64);
        x += lane >= off ? y : 0;
    }
    return x;
}

// block-wide exclusive scan of one int64 per thread (NT threads), returns the block total: wave
// scans, then every thread adds the totals of the waves before it (two barriers; the round-5
// Hillis-Steele form over LDS took 2 log2(NT) barriers)
template <int NT>
__device__ __forceinline__ int64_t block_excl_scan(int64_t x, int64_t& excl) {
    constexpr int NW = NT / 64;
    __shared__ int64_t ws[NW];
    const int w = threadIdx.x >> 6;
    const int64_t inc = wave_incl_scan(x);
    if ((threadIdx.x & 63) == 63) ws[w] = inc;
    __syncthreads();
    int64_t base = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        const int64_t v = ws[i];
        base += i < w ? v : 0;
        tot += v;
    }
    excl = base + inc - x;
    __syncthreads();   // ws is reused by the next scan
    return tot;
}

__global__ __launch_bounds__(kCmpThreads) void k_tile_sums(const int32_t* counts, int64_t n_ent,
                                                           int32_t capseg, int64_t* tile_kept,
                                                           int64_t* tile_raw) {
    int v[kCmpEpt];
    int64_t raw, kept, ex;
    const int64_t e0 = (int64_t)blockIdx.x * kCmpTile + (int64_t)threadIdx.x * kCmpEpt;
    load_counts(counts, n_ent, e0, capseg, v, raw, kept);
    const int64_t tk = block_excl_scan<kCmpThreads>(kept, ex);
    const int64_t tr = block_excl_scan<kCmpThreads>(raw, ex);
    if (threadIdx.x == 0) {
        tile_kept[blockIdx.x] = tk;
        tile_raw[blockIdx.x] = tr;
    }
}

// d_counts[0] = packets produced, d_counts[1] = packets stored in `out` (<= cap): written here,
// once per process call (the call's single compaction covers all of its sub-chunks), so the
// caller needs no zeroing launch.
__global__ __launch_bounds__(kScanThreads) void k_tile_scan(const int64_t* tile_kept, const int64_t* tile_raw,
                                                            int64_t ntiles, int64_t cap, int64_t* tile_off,
                                                            int64_t* d_counts) {
    const int64_t per = (ntiles + kScanThreads - 1) / kScanThreads;
    const int64_t b = threadIdx.x * per;
    int64_t sum = 0, sumw = 0;
    for (int64_t i = 0; i < per; ++i)
        if (b + i < ntiles) { sum += tile_raw[b + i]; sumw += tile_kept[b + i]; }
    int64_t run, ex;
    const int64_t w = block_excl_scan<kScanThreads>(sumw, run);
    const int64_t tot = block_excl_scan<kScanThreads>(sum, ex);
    for (int64_t i = 0; i < per; ++i)
        if (b + i < ntiles) { tile_off[b + i] = run; run += tile_kept[b + i]; }
    if (threadIdx.x == 0) {
        d_counts[0] = tot;
        d_counts[1] = w < cap ? w : cap;
    }
}

// ---- history roll: dst[i] = concat(old[0:hist_rows], fresh[0:fresh_rows])[fresh_rows + i] ----
__device__ __forceinline__ void hist_roll_part(uint8_t* dst, const uint8_t* old_hist, const uint8_t* fresh,
                                               int64_t hist_rows, int64_t fresh_rows, int64_t row_bytes,
                                               int64_t first, int64_t stride) {
    const int64_t total = hist_rows * row_bytes;
    for (int64_t b = first; b < total; b += stride) {
        const int64_t row = b / row_bytes, col = b % row_bytes;
        const int64_t src = fresh_rows + row;  // index into concat
        dst[b] = src < hist_rows ? old_hist[src * row_bytes + col]
                                 : fresh[(src - hist_rows) * row_bytes + col];
    }
}

// blocks [0, ntiles) gather; blocks after them run up to two history rolls (the call's raw-phase
// and ADC histories, which no kernel of the call reads: one launch fewer per call)
__global__ __launch_bounds__(kCmpThreads) void k_gather_events(const uint64_t* slots, const int32_t* counts,
                                                               int64_t n_ent, int32_t capseg,
                                                               const int64_t* tile_off, uint64_t* out,
                                                               int64_t cap, int ntiles, RollJob j1, int nb1,
                                                               RollJob j2) {
    if ((int)blockIdx.x >= ntiles) {
        const int rb = (int)blockIdx.x - ntiles;
        const bool first = rb < nb1;
        const RollJob& j = first ? j1 : j2;
        const int64_t b0 = first ? rb : rb - nb1;
        const int64_t nb = first ? nb1 : (int64_t)gridDim.x - ntiles - nb1;
        hist_roll_part((uint8_t*)j.dst, (const uint8_t*)j.old_hist, (const uint8_t*)j.fresh, j.hist_rows,
                       j.fresh_rows, j.row_bytes, b0 * blockDim.x + threadIdx.x, nb * blockDim.x);
        return;
    }
    int v[kCmpEpt];
    int64_t raw, kept, ex;
    const int64_t e0 = (int64_t)blockIdx.x * kCmpTile + (int64_t)threadIdx.x * kCmpEpt;
    load_counts(counts, n_ent, e0, capseg, v, raw, kept);
    block_excl_scan<kCmpThreads>(kept, ex);
    int64_t o = tile_off[blockIdx.x] + ex;
#pragma unroll
    for (int i = 0; i < kCmpEpt; ++i) {
        const uint64_t* src = slots + (e0 + i) * capseg;
        for (int k = 0; k < v[i]; ++k)
            if (o + k < cap) out[o + k] = src[k];
        o += v[i];
    }
}

static int roll_blocks(const RollJob* j) {
    if (!j) return 0;
    const int64_t total = j->hist_rows * j->row_bytes;
    const int64_t b = (total + 255) / 256;
    return (int)(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}

hipError_t launch_compact(const uint64_t* slots, const int32_t* counts, int64_t n_ent,
                          int32_t capseg, uint64_t* out, int64_t cap, int64_t* d_counts,
                          int64_t* scan_ws, const RollJob* roll1, const RollJob* roll2, hipStream_t s) {
    // scan_ws holds n_ent int64 (>= 3 per tile)
    const int64_t ntiles = (n_ent + kCmpTile - 1) / kCmpTile;
    int64_t* tile_kept = scan_ws;
    int64_t* tile_raw = scan_ws + ntiles;
    int64_t* tile_off = scan_ws + 2 * ntiles;
    hipLaunchKernelGGL(k_tile_sums, dim3((unsigned)ntiles), dim3(kCmpThreads), 0, s, counts, n_ent, capseg,
                       tile_kept, tile_raw);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(kScanThreads), 0, s, tile_kept, tile_raw, ntiles, cap,
                       tile_off, d_counts);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const int nb1 = roll_blocks(roll1), nb2 = roll_blocks(roll2);
    const RollJob none{};
    hipLaunchKernelGGL(k_gather_events, dim3((unsigned)(ntiles + nb1 + nb2)), dim3(kCmpThreads), 0, s, slots,
                       counts, n_ent, capseg, tile_off, out, cap, (int)ntiles, roll1 ? *roll1 : none, nb1,
                       roll2 ? *roll2 : none);
    return hipGetLastError();
}

__global__ void k_hist_roll(uint8_t* dst, const uint8_t* old_hist, const uint8_t* fresh,
                            int64_t hist_rows, int64_t fresh_rows, int64_t row_bytes) {
    hist_roll_part(dst, old_hist, fresh, hist_rows, fresh_rows, row_bytes,
                   (int64_t)blockIdx.x * blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x);
}

hipError_t launch_hist_roll(void* dst, const void* old_hist, const void* fresh, int64_t hist_rows,
                            int64_t fresh_rows, int64_t row_bytes, hipStream_t s) {
    const int64_t total = hist_rows * row_bytes;
    const int blocks = (int)((total + 255) / 256 < 1024 ? (total + 255) / 256 : 1024);
    hipLaunchKernelGGL(k_hist_roll, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, s, (uint8_t*)dst,
                       (const uint8_t*)old_hist, (const uint8_t*)fresh, hist_rows, fresh_rows,
                       row_bytes);
    return hipGetLastError();
}

}  // namespace mkid
