// C ABI of libmkidgpu.so (include/mkidgpu.h): context, configuration, streaming process calls.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <utility>
#include <atomic>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "mkid_internal.h"
#include "mkid_plan.h"

using namespace mkid;

namespace {

// error text of a failed mkid_create (no context yet); per thread, so that contexts created
// concurrently from several host threads do not overwrite each other's message
thread_local std::string g_err;

// Default IQ low-pass: LUT/BlackmanFilter_250kHz.txt quantised as int(x*(2**11-1))
// (ROACH_Pulses.py:69, 88; importFIRcoeffs default ROACH_Pulses.py:1101).
const int16_t kBlackman250k[kFirTaps] = {0,   0,   3,   8,   17,  32,  53,  80,  111, 142, 172, 194, 206,
                                         206, 194, 172, 142, 111, 80,  53,  32,  17,  8,   3,   0,   0};

struct KTime {
    int k;
    hipEvent_t a, b;
};

using plan::kSegL;
using plan::kSvfW;
using plan::seg_capacity;
using plan::SubPlan;

}  // namespace

struct mkid_ctx {
    mkid_cfg cfg{};
    int device = 0;
    hipStream_t own = nullptr, stream = nullptr;
    std::string err;
    int C = 0, N = 0, M = 0, T = 0, P = 0, capc = 0;
    int ncu = 256;  // compute units of the device (launch grids are per-CU multiples)
    // what the carried stream state belongs to: 0 none (fresh / reset), 1 an ADC stream
    // (mkid_process*), 2 a phase-row stream (mkid_trigger_phase); mixing them needs a reset
    int stream_kind = 0;
    int64_t Kmax = 0, Jmax = 0;
    // configuration
    float* d_pfb = nullptr;      // effective taps h_q 2^-S (float, split path)
    uint2* d_pfbq = nullptr;     // [N] {h_q[0]|h_q[1]<<16, h_q[2]|h_q[3]<<16} (fused path, int16 dot2)
    int pfb_shift = 0;           // S
    int32_t* d_bins = nullptr;
    float2* d_lo = nullptr;
    int16_t* d_fir = nullptr;
    // IQ-loop centres (loadIQcenters) and the centred low-pass constants derived from them and the
    // low-pass taps (upload_centring): d_ncen = -c', d_cor = r (mkid_internal.h Centring)
    std::vector<float> h_ic, h_qc;
    float2 *d_ncen = nullptr, *d_cor = nullptr;
    std::vector<double> h_gc;   // [2C] G c' (= r + c): added back to y' for the raw IQ
    int32_t* d_thr = nullptr;
    int32_t* d_rearm = nullptr;      // [C] re-arm levels (upload_rearm)
    std::vector<int32_t> h_thr;
    int32_t rearm_q8 = 0;            // mkid_set_rearm hysteresis fraction (/256)
    LpfTaps lpf{};
    int32_t mode = MKID_BASE_EMA, alpha = 41, kf = 82, kq = 93623, base_thr = 8192;
    // stream state
    uint32_t *d_xhist = nullptr, *d_xtmp = nullptr;
    float2 *d_zhist = nullptr, *d_ztmp = nullptr;
    int16_t *d_rhist = nullptr, *d_rtmp = nullptr;
    TrigState* d_tstate = nullptr;
    int64_t k0 = 0, j0 = 0;
    // two-stream pipeline: stream A (= `stream`) runs the channeliser, stream B the low-pass,
    // trigger and compaction of the previous sub-chunk; z is double-buffered between them.
    hipStream_t sB = nullptr;
    hipEvent_t ev_zready[2] = {nullptr, nullptr}, ev_zfree[2] = {nullptr, nullptr};
    hipEvent_t ev_start = nullptr, ev_done = nullptr;
    int zi = 0;
    int64_t G = 0;  // pipeline sub-chunk (samples)
    // test hook (MKID_FAULT_LAUNCH=n at mkid_create): the n-th front-end launch of the context
    // reports a HIP failure after it was enqueued, to test the state a partly enqueued call leaves
    int64_t fault_launch = 0, launch_count = 0;
    int64_t last_raw_row = 0;       // first row of the last sub-chunk's raw phase in d_raw
    bool fused = false;  // K1-K6 in one kernel (k_front / k_front3 / k_front5: no z buffers, no stream B work)
    int64_t H = 0;       // ADC history samples carried between calls
    // workspace
    float2* d_zb[2] = {nullptr, nullptr};
    int16_t* d_raw = nullptr;
    int16_t* d_filt = nullptr;      // [Jmax][C] SVF filter pre-pass output (k_mf_rows)
    RefixRes* d_refix = nullptr;    // [C][nsub_max * nseg_max] SVF parallel re-run results (k_trig_refix)
    uint64_t* d_refix_pk = nullptr; // [slot_cap] their true packets (the slot table's geometry)
    long long* d_ysum = nullptr;   // [C][2] fixed point 2^-kYsumFrac: sums of y' while armed
    // avgIQ accumulator (K9; startAccumulator / avgIQ_ctrl, ROACH_Setup.py:654-659): armed by
    // mkid_set_accumulator; rows accumulated since arming and the host-side sums of G c' over them
    bool acc_on = false;
    int64_t acc_rows = 0;
    std::vector<double> acc_off;   // [2C]
    uint64_t* d_slots = nullptr;     // [C][nseg][capseg]
    int32_t* d_chcounts = nullptr;   // [C][nseg]
    int64_t* d_scan = nullptr;       // [C][nseg]
    TrigState *d_sspec = nullptr, *d_send = nullptr;  // [nseg][C]
    uint64_t* d_scratch = nullptr;   // [C][capseg]
    int32_t* d_reruns = nullptr;     // [C]
    int64_t nseg_max = 0, slot_cap = 0, scratch_cap = 0, trig_slots = 0;
    int64_t svf_lanes = 65536, svf_w = kSvfW;  // SVF segmentation (plan_sub)
    int64_t nsub_max = 0;    // sub-chunks per call (ceil(max_chunk / G))
    plan::Workspace ws;      // what the context was sized for (plan::size_workspace)
    int64_t* d_counts = nullptr;  // [2] used by the host-pointer API
    int64_t last_J = 0;     // phase rows of the last call
    int64_t last_subJ = 0;  // rows of its last sub-chunk (held in d_raw)
    // IQ snapshot tap: low-pass output of one channel for the rows of the last call
    int32_t iq_ch = -1;
    int16_t* d_iqtap = nullptr;     // [max_chunk/N][2]
    float* d_hcoeff = nullptr;      // [C][h_ncoeff] pulse-height filter (mkid_set_pulse_filter)
    int32_t h_ncoeff = 0, h_pre = 0;
    float *d_phist = nullptr, *d_phist_tmp = nullptr;  // [h_ncoeff][C] last phase rows seen by pulse_heights
    int64_t phist_end = -1, phist_rows = 0;          // global row after its last row; valid rows
    int64_t iq_rows = 0;
    // host copies behind the folded LO table (d_lo = conj(LUT)/2^15 with the (-1)^(b (k+1))
    // bin-parity sign of K4 folded in: P is even, so the sign depends on k mod P only)
    std::vector<float2> h_lo;      // [P][C]
    std::vector<int32_t> h_bins;   // [C]
    // select-slot order of the N = 2048 front end (k_front3): d_slot_ch[slot] = channel (slot_order
    // below; MKID_SLOT_ORDER=0 keeps the identity)
    int16_t* d_slot_ch = nullptr;
    bool slot_order_on = true;
    // replay-trigger workspace (lazy, grown on demand)
    uint32_t* d_rflags = nullptr;
    double* d_rmeans = nullptr;
    size_t rflags_n = 0, rmeans_n = 0;
    // host-API staging (lazy)
    uint32_t* d_in = nullptr;
    float* d_phase_ws = nullptr;
    uint64_t* d_ev_ws = nullptr;
    // timing
    bool timing = false;
    uint32_t timing_mask = 0;   // bit k: kernel k is timed
    std::vector<KTime> pending;
    std::vector<hipEvent_t> pool;
    double tot_ms[MKID_K_COUNT] = {0};
    int64_t launches[MKID_K_COUNT] = {0};
};

#define FAIL(ctx, code, msg)       \
    do {                           \
        (ctx)->err = (msg);        \
        return (code);             \
    } while (0)

#define HIPCHK(ctx, call)                                                                  \
    do {                                                                                   \
        hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess) {                                                            \
            (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e_);               \
            return MKID_E_HIP;                                                             \
        }                                                                                  \
    } while (0)

static hipEvent_t get_event(mkid_ctx* c) {
    if (!c->pool.empty()) {
        hipEvent_t e = c->pool.back();
        c->pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

static void tstart(mkid_ctx* c, int k, KTime* kt, hipStream_t s) {
    kt->k = -1;
    if (!c->timing || !((c->timing_mask >> k) & 1u)) return;
    kt->a = get_event(c);
    kt->b = get_event(c);
    if (!kt->a || !kt->b) return;
    kt->k = k;
    (void)hipEventRecord(kt->a, s);
}

static void tstop(mkid_ctx* c, KTime* kt, hipStream_t s) {
    if (kt->k < 0) return;
    (void)hipEventRecord(kt->b, s);
    c->pending.push_back(*kt);
}

static int flush_timing(mkid_ctx* c) {
    for (auto& kt : c->pending) {
        HIPCHK(c, hipEventSynchronize(kt.b));
        float ms = 0.f;
        HIPCHK(c, hipEventElapsedTime(&ms, kt.a, kt.b));
        c->tot_ms[kt.k] += ms;
        c->launches[kt.k] += 1;
        c->pool.push_back(kt.a);
        c->pool.push_back(kt.b);
    }
    c->pending.clear();
    return MKID_OK;
}

static void free_all(mkid_ctx* c) {
    void* ptrs[] = {c->d_pfb,   c->d_pfbq,  c->d_bins,  c->d_lo,    c->d_fir,    c->d_ncen,   c->d_cor,
                    c->d_thr,   c->d_rearm, c->d_xhist, c->d_xtmp,  c->d_zhist,  c->d_ztmp,   c->d_rhist,
                    c->d_rtmp,  c->d_tstate, c->d_zb[0], c->d_zb[1], c->d_raw, c->d_filt, c->d_ysum, c->d_slots,
                    c->d_chcounts, c->d_scan, c->d_counts, c->d_in,  c->d_phase_ws, c->d_ev_ws,
                    c->d_sspec, c->d_send,  c->d_scratch, c->d_reruns, c->d_rflags, c->d_rmeans, c->d_iqtap, c->d_hcoeff,
                    c->d_phist, c->d_phist_tmp, c->d_slot_ch, c->d_refix, c->d_refix_pk};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (auto& kt : c->pending) {
        (void)hipEventDestroy(kt.a);
        (void)hipEventDestroy(kt.b);
    }
    for (auto e : c->pool) (void)hipEventDestroy(e);
    hipEvent_t evs[] = {c->ev_zready[0], c->ev_zready[1], c->ev_zfree[0], c->ev_zfree[1], c->ev_start, c->ev_done};
    for (auto e : evs)
        if (e) (void)hipEventDestroy(e);
    if (c->sB) (void)hipStreamDestroy(c->sB);
    if (c->own) (void)hipStreamDestroy(c->own);
}

template <typename T>
static hipError_t dalloc(T** p, size_t n) {
    return hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(T));
}

static void default_pfb(int N, int T, std::vector<float>& h) {
    const int L = T * N;
    std::vector<double> d(L);
    double s = 0;
    for (int n = 0; n < L; ++n) {
        const double x = (n - (L - 1) / 2.0) / N;
        const double sinc = x == 0 ? 1.0 : std::sin(M_PI * x) / (M_PI * x);
        d[n] = sinc * (0.54 - 0.46 * std::cos(2 * M_PI * n / (L - 1)));
        s += d[n];
    }
    h.resize(L);
    for (int n = 0; n < L; ++n) h[n] = (float)(d[n] / s);
}

// scoped device allocations for the (non-hot-path) template calls
struct DevBufs {
    std::vector<void*> p;
    ~DevBufs() { for (void* q : p) (void)hipFree(q); }
    template <typename T>
    hipError_t get(T** out, size_t n) {
        void* q = nullptr;
        hipError_t e = hipMalloc(&q, std::max<size_t>(n, 1) * sizeof(T));
        if (e == hipSuccess) p.push_back(q);
        *out = (T*)q;
        return e;
    }
};

using plan::quantize_pfb;

static int upload_lo_folded(mkid_ctx* c);
static int upload_slot_order(mkid_ctx* c);
static int upload_centring(mkid_ctx* c);
static int upload_pfb(mkid_ctx* c, const float* coeffs);

extern "C" {

const char* mkid_global_error(void) { return g_err.c_str(); }

int mkid_default_cfg(mkid_cfg* cfg, int32_t n_channels) {
    if (!cfg || n_channels <= 0 || 65536 % n_channels != 0) return MKID_E_ARG;
    std::memset(cfg, 0, sizeof(*cfg));
    cfg->n_channels = n_channels;
    cfg->fft_len = 2 * n_channels;
    cfg->pfb_taps = kPfbTaps;
    cfg->fir_taps = kFirTaps;
    cfg->dds_entries = 65536 / n_channels;
    cfg->dead_time = 32;
    cfg->max_events_per_ch = 0;
    cfg->max_chunk = (int64_t)1 << 22;
    cfg->sample_rate = 512e6;
    return MKID_OK;
}

int mkid_create(const mkid_cfg* cfg, int32_t device, mkid_ctx** out) {
    if (!cfg || !out) { g_err = "null argument"; return MKID_E_ARG; }
    *out = nullptr;
    const int C = cfg->n_channels, N = cfg->fft_len;
    if (N != 2 * C || !channelize_supported(N)) { g_err = "unsupported geometry: need N = 2C, N in {128..4096}"; return MKID_E_ARG; }
    if (cfg->pfb_taps != kPfbTaps || cfg->fir_taps != kFirTaps) { g_err = "pfb_taps must be 4 and fir_taps 26"; return MKID_E_ARG; }
    const int P = cfg->dds_entries;
    if (P < 2 || (P & (P - 1)) != 0) { g_err = "dds_entries must be a power of two >= 2"; return MKID_E_ARG; }
    if (cfg->max_chunk < N || cfg->max_chunk % N != 0) { g_err = "max_chunk must be a positive multiple of N"; return MKID_E_ARG; }
    if (cfg->dead_time < 0) { g_err = "dead_time < 0"; return MKID_E_ARG; }
    if (cfg->front != MKID_FRONT_AUTO && cfg->front != MKID_FRONT_SPLIT) { g_err = "bad front mode"; return MKID_E_ARG; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) { g_err = "no HIP device"; return MKID_E_NODEV; }
    if (device < 0 || device >= ndev) { g_err = "bad device index"; return MKID_E_ARG; }
    mkid_ctx* c = new (std::nothrow) mkid_ctx();
    if (!c) { g_err = "out of host memory"; return MKID_E_ARG; }
    c->cfg = *cfg;
    c->device = device;
    c->C = C; c->N = N; c->M = N / 2; c->T = kPfbTaps; c->P = P;
    c->fused = cfg->front == MKID_FRONT_AUTO && fused_supported(N);
    {
        const char* so = getenv("MKID_SLOT_ORDER");
        c->slot_order_on = !(so && atoi(so) == 0);
        if (const char* fl = getenv("MKID_FAULT_LAUNCH")) c->fault_launch = atoll(fl);
    }
    int64_t trig_slots = trigger_wave_slots(device);
    // tuning/test knob: pretend the GPU holds this many trigger waves (forces longer segments)
    if (const char* ev = getenv("MKID_TRIG_WAVE_SLOTS")) trig_slots = std::max<int64_t>(1, atoll(ev));
    int64_t svf_lanes = 0, svf_w = kSvfW;
    {   // SVF segments: one per SIMD lane (4 SIMDs x 64 lanes per CU, round 6); test/tuning knobs
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu <= 0)
            ncu = 256;
        c->ncu = ncu;
        svf_lanes = (int64_t)ncu * 256;
        if (const char* ev = getenv("MKID_SVF_LANES")) svf_lanes = std::max<int64_t>(1, atoll(ev));
        if (const char* ev = getenv("MKID_SVF_WARMUP"))
            svf_w = std::max<int64_t>(1, atoll(ev) / kFirTaps) * kFirTaps;
    }
    if (const char* msg = plan::size_workspace(*cfg, c->fused, trig_slots, svf_lanes, svf_w, c->ws)) {
        g_err = msg;
        delete c;
        return MKID_E_ARG;
    }
    c->G = c->ws.G;
    c->Kmax = c->ws.Kmax;
    c->Jmax = c->ws.Jmax;
    c->nsub_max = c->ws.nsub_max;
    c->capc = (int)c->ws.capc;
    c->trig_slots = c->ws.trig_slots;
    c->svf_lanes = c->ws.svf_lanes;
    c->svf_w = c->ws.svf_w;
    c->nseg_max = c->ws.nseg_max;
    c->slot_cap = c->ws.slot_cap;
    c->scratch_cap = c->ws.scratch_cap;
    c->H = c->fused ? front_hist_samples(N) : (int64_t)c->T * N - c->M;
    const int64_t H = c->H;
    auto fail = [&](hipError_t e, const char* what) {
        g_err = std::string(what) + ": " + hipGetErrorString(e);
        free_all(c);
        delete c;
        return MKID_E_HIP;
    };
    hipError_t e;
#define AL(p, n) if ((e = dalloc(&c->p, (n))) != hipSuccess) return fail(e, "hipMalloc " #p)
    if ((e = hipSetDevice(device)) != hipSuccess) return fail(e, "hipSetDevice");
    if ((e = hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking)) != hipSuccess) return fail(e, "hipStreamCreate");
    c->stream = c->own;
    if ((e = hipStreamCreateWithFlags(&c->sB, hipStreamNonBlocking)) != hipSuccess) return fail(e, "hipStreamCreate B");
    for (hipEvent_t* ev : {&c->ev_zready[0], &c->ev_zready[1], &c->ev_zfree[0], &c->ev_zfree[1], &c->ev_start, &c->ev_done})
        if ((e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess) return fail(e, "hipEventCreate");
    for (int b = 0; b < 2; ++b)
        if ((e = hipEventRecord(c->ev_zfree[b], c->sB)) != hipSuccess) return fail(e, "hipEventRecord");
    AL(d_pfb, (size_t)c->T * N);
    AL(d_pfbq, (size_t)N);
    AL(d_bins, C);
    AL(d_lo, (size_t)C * P);
    AL(d_fir, (size_t)C * kFirTaps);
    AL(d_ncen, C);
    AL(d_cor, C);
    AL(d_thr, C);
    AL(d_rearm, C);
    AL(d_xhist, H);
    AL(d_xtmp, H);
    AL(d_zhist, (size_t)kLpfHist * C);
    AL(d_ztmp, (size_t)kLpfHist * C);
    AL(d_rhist, (size_t)kRawHist * C);
    AL(d_rtmp, (size_t)kRawHist * C);
    AL(d_tstate, C);
    if (!c->fused) {
        AL(d_zb[0], (size_t)c->Kmax * C);
        AL(d_zb[1], (size_t)c->Kmax * C);
    }
    AL(d_raw, (size_t)c->Jmax * C);
    AL(d_iqtap, (size_t)(cfg->max_chunk / N) * 2);
    AL(d_ysum, (size_t)2 * C);
    AL(d_slots, (size_t)c->slot_cap);
    AL(d_chcounts, (size_t)C * c->nsub_max * c->nseg_max);
    AL(d_scan, (size_t)C * c->nsub_max * c->nseg_max + 64);  // >= 3 int64 per compaction tile
    AL(d_sspec, (size_t)C * c->nseg_max);
    AL(d_send, (size_t)C * c->nseg_max);
    AL(d_scratch, (size_t)C * c->scratch_cap);
    AL(d_reruns, C);
    AL(d_counts, 2);
    AL(d_slot_ch, C);
#undef AL
    // defaults: identity bins, unit LO, Blackman 250 kHz low-pass, zero matched filter (no
    // triggers), zero centres, thresholds off, EMA baseline alpha=41 gate=8192.
    std::vector<float> h;
    default_pfb(N, c->T, h);
    std::vector<int32_t> bins(C), thr(C, INT_MIN / 2);
    for (int i = 0; i < C; ++i) bins[i] = i;
    std::vector<float2> lo((size_t)C * P, make_float2(32767.f / 32768.f, 0.f));
    std::vector<int16_t> fir((size_t)C * kFirTaps, 0);
    for (int i = 0; i < kFirTaps; ++i) c->lpf.g[i] = kBlackman250k[i] / 2048.0f;
    c->h_thr = thr;
    c->h_ic.assign(C, 0.f);
    c->h_qc.assign(C, 0.f);
    c->acc_off.assign(2 * (size_t)C, 0.0);
    if ((e = hipMemcpy(c->d_bins, bins.data(), C * 4, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(c->d_thr, thr.data(), C * 4, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(c->d_rearm, thr.data(), C * 4, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(c->d_lo, lo.data(), lo.size() * 8, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(c->d_fir, fir.data(), fir.size() * 2, hipMemcpyHostToDevice)) != hipSuccess)
        return fail(e, "hipMemcpy defaults");
    c->h_lo = lo;
    c->h_bins = bins;
    *out = c;
    if (upload_pfb(c, h.data()) != MKID_OK || upload_slot_order(c) != MKID_OK || upload_centring(c) != MKID_OK ||
        mkid_reset_stream(c) != MKID_OK) {
        g_err = c->err;
        free_all(c);
        delete c;
        *out = nullptr;
        return MKID_E_HIP;
    }
    return MKID_OK;
}

int mkid_destroy(mkid_ctx* c) {
    if (!c) return MKID_E_ARG;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    free_all(c);
    delete c;
    return MKID_OK;
}

const char* mkid_last_error(const mkid_ctx* c) { return c ? c->err.c_str() : g_err.c_str(); }

int mkid_get_cfg(const mkid_ctx* c, mkid_cfg* out) {
    if (!c || !out) return MKID_E_ARG;
    *out = c->cfg;
    return MKID_OK;
}

int mkid_set_stream(mkid_ctx* c, void* s) {
    if (!c) return MKID_E_ARG;
    c->stream = s ? (hipStream_t)s : c->own;
    return MKID_OK;
}

static int upload(mkid_ctx* c, void* dst, const void* src, size_t bytes) {
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return MKID_OK;
}

static int upload_pfb(mkid_ctx* c, const float* coeffs) {
    const int T = c->T, N = c->N;
    std::vector<int16_t> hq;
    const int S = quantize_pfb(coeffs, T, N, hq);
    std::vector<float> hf(hq.size());
    for (size_t i = 0; i < hq.size(); ++i) hf[i] = (float)std::ldexp((double)hq[i], -S);
    std::vector<uint2> hp(N);
    for (int p = 0; p < N; ++p) {
        auto u16 = [&](int t) { return (uint32_t)(uint16_t)hq[(size_t)t * N + p]; };
        hp[p] = make_uint2(u16(0) | (u16(1) << 16), u16(2) | (u16(3) << 16));
    }
    int r = upload(c, c->d_pfb, hf.data(), hf.size() * 4);
    if (r) return r;
    r = upload(c, c->d_pfbq, hp.data(), hp.size() * 8);
    if (r) return r;
    c->pfb_shift = S;
    return upload_lo_folded(c);  // the fused path folds 2^-S into the LO table
}

int mkid_pfb_effective_taps(const float* coeffs, int32_t T, int32_t N, float* out, int32_t* shift) {
    if (!coeffs || !out || T <= 0 || N <= 0) return MKID_E_ARG;
    std::vector<int16_t> hq;
    const int S = quantize_pfb(coeffs, T, N, hq);
    for (size_t i = 0; i < hq.size(); ++i) out[i] = (float)std::ldexp((double)hq[i], -S);
    if (shift) *shift = S;
    return MKID_OK;
}

int mkid_set_pfb(mkid_ctx* c, const float* coeffs, int32_t n) {
    if (!c || !coeffs) return MKID_E_ARG;
    if (n != c->T * c->N) FAIL(c, MKID_E_ARG, "pfb coefficient count must be T*N");
    return upload_pfb(c, coeffs);
}

int mkid_set_bins(mkid_ctx* c, const int32_t* bins, int32_t n) {
    if (!c || !bins) return MKID_E_ARG;
    if (n != c->C) FAIL(c, MKID_E_ARG, "need one bin per channel");
    std::vector<int32_t> b(bins, bins + n);
    for (auto& v : b) v = ((v % c->N) + c->N) % c->N;
    int r = upload(c, c->d_bins, b.data(), (size_t)n * 4);
    if (r) return r;
    c->h_bins = b;
    r = upload_slot_order(c);
    if (r) return r;
    return upload_lo_folded(c);
}

int mkid_set_dds(mkid_ctx* c, const int16_t* li, const int16_t* lq, int32_t P) {
    if (!c || !li || !lq) return MKID_E_ARG;
    if (P != c->P) FAIL(c, MKID_E_ARG, "entries_per_ch must equal cfg.dds_entries");
    // device layout [P][C] (input is [C][P]): one frame reads one contiguous row
    std::vector<float2> lo((size_t)c->C * P);
    for (int ch = 0; ch < c->C; ++ch)
        for (int p = 0; p < P; ++p) {
            const size_t i = (size_t)ch * P + p;
            lo[(size_t)p * c->C + ch] = make_float2(li[i] / 32768.f, -lq[i] / 32768.f);
        }
    c->h_lo = std::move(lo);
    return upload_lo_folded(c);
}

// k_front3 select-slot order: plan::slot_order (mkid_plan.cpp)
using plan::slot_order;

static int upload_slot_order(mkid_ctx* c) {
    std::vector<int16_t> so;
    if (c->slot_order_on) {
        slot_order(c->h_bins, c->C, so);
    } else {
        so.resize(c->C);
        for (int i = 0; i < c->C; ++i) so[i] = (int16_t)i;
    }
    return upload(c, c->d_slot_ch, so.data(), so.size() * 2);
}

int mkid_slot_order(const int32_t* bins, int32_t C, int16_t* out) {
    if (!bins || !out || C <= 0) return MKID_E_ARG;
    std::vector<int32_t> b(bins, bins + C);
    std::vector<int16_t> so;
    slot_order(b, C, so);
    std::copy(so.begin(), so.end(), out);
    return MKID_OK;
}

// d_lo[p][c] = h_lo[p][c] * (-1)^(b_c (k+1)) for any frame k = p (mod P): odd bins flip the sign
// on even rows (P is even). The kernels then multiply by d_lo only.
static int upload_lo_folded(mkid_ctx* c) {
    std::vector<float2> lo = c->h_lo;
    // fused path: the PFB output is the integer h_q . x, so the 2^-S tap scale joins the LO
    const float sc = c->fused ? (float)std::ldexp(1.0, -c->pfb_shift) : 1.0f;
    for (int p = 0; p < c->P; ++p)
        for (int ch = 0; ch < c->C; ++ch) {
            float2& v = lo[(size_t)p * c->C + ch];
            const float sg = ((p & 1) == 0 && (c->h_bins[ch] & 1)) ? -sc : sc;
            v = make_float2(v.x * sg, v.y * sg);
        }
    return upload(c, c->d_lo, lo.data(), lo.size() * 8);
}

int mkid_set_lpf(mkid_ctx* c, const int16_t* taps, int32_t n) {
    if (!c || !taps) return MKID_E_ARG;
    if (n != kFirTaps) FAIL(c, MKID_E_ARG, "low-pass must have 26 taps");
    for (int i = 0; i < n; ++i) c->lpf.g[i] = taps[i] / 2048.0f;
    return upload_centring(c);   // c' = c / G depends on the taps' sum G
}

// Centred low-pass constants (mkid_internal.h Centring): G = sum_i g_i (exact: g_i = k_i / 2^11),
// c' = fp32(c / G), r = fp32(G c' - c) evaluated in float64 (G c' is exact there: 16 x 24 bits), so
// y' + r = y - c up to the rounding of r (|r| ~ 2^-24 |c|). |G| < kCentringMinGain (taps with a
// small DC gain, all-zero taps): c' = 0, r = -c, the uncentred form — c' = c / G would grow as 1 / G
// and the low-pass accumulation's fp32 rounding with it.
static constexpr double kCentringMinGain = 0.25;
static int upload_centring(mkid_ctx* c) {
    double G = 0.0;
    for (int i = 0; i < kFirTaps; ++i) G += (double)c->lpf.g[i];
    const bool centred = std::fabs(G) >= kCentringMinGain;
    std::vector<float2> nc((size_t)c->C), cr((size_t)c->C);
    c->h_gc.assign(2 * (size_t)c->C, 0.0);
    for (int ch = 0; ch < c->C; ++ch) {
        const double ci = c->h_ic[ch], cq = c->h_qc[ch];
        const float pi = centred ? (float)(ci / G) : 0.f, pq = centred ? (float)(cq / G) : 0.f;
        nc[ch] = make_float2(-pi, -pq);
        cr[ch] = make_float2((float)(G * pi - ci), (float)(G * pq - cq));
        c->h_gc[2 * ch] = G * pi;
        c->h_gc[2 * ch + 1] = G * pq;
    }
    int r = upload(c, c->d_ncen, nc.data(), nc.size() * 8);
    return r ? r : upload(c, c->d_cor, cr.data(), cr.size() * 8);
}

// r + c of the IQ-tap channel (the tap reports y = y' + r + c)
static float2 tap_offset(const mkid_ctx* c) {
    if (c->iq_ch < 0) return make_float2(0.f, 0.f);
    return make_float2((float)c->h_gc[2 * c->iq_ch], (float)c->h_gc[2 * c->iq_ch + 1]);
}

// the avgIQ accumulator after an armed call of J rows: the device summed y', the host adds J G c'.
// acc_rows < 0: a failed call left partial sums; the average stays invalid until re-armed.
static void acc_account(mkid_ctx* c, int64_t J) {
    if (!c->acc_on || c->acc_rows < 0) return;
    c->acc_rows += J;
    for (size_t i = 0; i < c->acc_off.size(); ++i) c->acc_off[i] += (double)J * c->h_gc[i];
}

int mkid_set_fir(mkid_ctx* c, const int16_t* taps, int32_t nch, int32_t nt) {
    if (!c || !taps) return MKID_E_ARG;
    if (nch != c->C || nt != kFirTaps) FAIL(c, MKID_E_ARG, "matched filter must be [C][26]");
    for (int64_t i = 0; i < (int64_t)nch * nt; ++i)
        if (taps[i] < -2048 || taps[i] > 2047) FAIL(c, MKID_E_ARG, "matched-filter tap outside 12-bit range");
    return upload(c, c->d_fir, taps, (size_t)nch * nt * 2);
}

int mkid_set_centers(mkid_ctx* c, const float* ic, const float* qc, int32_t n) {
    if (!c || !ic || !qc) return MKID_E_ARG;
    if (n != c->C) FAIL(c, MKID_E_ARG, "need one centre per channel");
    for (int i = 0; i < n; ++i)
        if (!std::isfinite(ic[i]) || !std::isfinite(qc[i])) FAIL(c, MKID_E_ARG, "centres must be finite");
    c->h_ic.assign(ic, ic + n);
    c->h_qc.assign(qc, qc + n);
    return upload_centring(c);
}

// re-arm levels from the thresholds and the hysteresis fraction (plan::rearm_level)
static int upload_rearm(mkid_ctx* c) {
    std::vector<int32_t> lv(c->h_thr.size());
    for (size_t i = 0; i < lv.size(); ++i) lv[i] = plan::rearm_level(c->h_thr[i], c->rearm_q8);
    return upload(c, c->d_rearm, lv.data(), lv.size() * 4);
}

int mkid_set_thresholds(mkid_ctx* c, const int32_t* thr, int32_t n) {
    if (!c || !thr) return MKID_E_ARG;
    if (n != c->C) FAIL(c, MKID_E_ARG, "need one threshold per channel");
    int r = upload(c, c->d_thr, thr, (size_t)n * 4);
    if (r) return r;
    c->h_thr.assign(thr, thr + n);
    return upload_rearm(c);
}

int mkid_set_rearm(mkid_ctx* c, int32_t frac_q8) {
    if (!c) return MKID_E_ARG;
    if (frac_q8 < 0 || frac_q8 > 256) FAIL(c, MKID_E_ARG, "re-arm fraction must be 0..256 (/256)");
    c->rearm_q8 = frac_q8;
    return upload_rearm(c);
}

int mkid_set_baseline(mkid_ctx* c, int32_t mode, int32_t alpha, int32_t kf, int32_t kq, int32_t base_thr) {
    if (!c) return MKID_E_ARG;
    if (mode < MKID_BASE_NONE || mode > MKID_BASE_SVF) FAIL(c, MKID_E_ARG, "bad baseline mode");
    // Fix12_9; above 2.0 (1024) the EMA diverges and its int32 arithmetic overflows
    if (alpha < 0 || alpha > 1024) FAIL(c, MKID_E_ARG, "alpha must be Fix12_9 in 0..1024 (gain <= 2.0)");
    if (kf < 0 || kf >= (1 << 18) || kq < 0 || kq >= (1 << 18)) FAIL(c, MKID_E_ARG, "kf/kq must be Fix18_16");
    if (base_thr < 0 || base_thr > 65535) FAIL(c, MKID_E_ARG, "base_thr must be Fix16_13 (0..65535)");
    if (mode == MKID_BASE_SVF && !c->d_filt) {   // the SVF filter pre-pass rows, allocated on first use
        HIPCHK(c, hipSetDevice(c->device));
        HIPCHK(c, dalloc(&c->d_filt, (size_t)c->Jmax * c->C));
        // and the parallel re-run tables (k_trig_refix): one result per slot-table segment, one
        // packet table the size of the slot table. Both or neither (without them the fix-up walks
        // the failed segments in the channel's wave, k_trig_fix)
        RefixRes* rf = nullptr;
        uint64_t* rp = nullptr;
        hipError_t e = dalloc(&rf, (size_t)c->C * (size_t)c->ws.nsub_max * (size_t)std::max<int64_t>(1, c->ws.nseg_max));
        if (e == hipSuccess) e = dalloc(&rp, (size_t)c->slot_cap);
        if (e != hipSuccess) {
            if (rf) (void)hipFree(rf);
            FAIL(c, MKID_E_HIP, "hipMalloc of the SVF re-run tables failed");
        }
        c->d_refix = rf;
        c->d_refix_pk = rp;
    }
    c->mode = mode; c->alpha = alpha; c->kf = kf; c->kq = kq; c->base_thr = base_thr;
    return MKID_OK;
}

int mkid_reset_stream(mkid_ctx* c) {
    if (!c) return MKID_E_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->sB));
    HIPCHK(c, hipMemsetAsync(c->d_xhist, 0, (size_t)c->H * 4, c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_zhist, 0, (size_t)kLpfHist * c->C * 8, c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_rhist, 0, (size_t)kRawHist * c->C * 2, c->stream));
    {   // start-of-stream hold-off: DEAD for kHoldOff samples, no baseline (trig_common.h)
        std::vector<TrigState> st0((size_t)c->C, TrigState{0, 0, 2 /*ST_DEAD*/, kHoldOff, 0, 0, 0, 0, 0, 0});
        HIPCHK(c, hipMemcpyAsync(c->d_tstate, st0.data(), st0.size() * sizeof(TrigState), hipMemcpyHostToDevice,
                                 c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    HIPCHK(c, hipMemsetAsync(c->d_ysum, 0, (size_t)c->C * 16, c->stream));   // avgIQ: sums restart
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->acc_rows = 0;
    std::fill(c->acc_off.begin(), c->acc_off.end(), 0.0);
    c->k0 = 0;
    c->j0 = 0;
    c->stream_kind = 0;
    c->last_J = 0;
    c->last_subJ = 0;
    c->last_raw_row = 0;
    c->phist_end = -1;     // pulse-height phase history: a reset starts a new stream
    c->phist_rows = 0;
    return MKID_OK;
}

// The call's trigger plan (plan::plan_call, mkid_plan.cpp) within the context's workspace.
static int plan_call(mkid_ctx* c, int64_t n, std::vector<SubPlan>& subs, int32_t& stride, int32_t& capseg) {
    if (const char* msg = plan::plan_call(c->ws, c->C, c->N, c->mode, c->cfg.dead_time, n, subs, stride, capseg))
        FAIL(c, MKID_E_ARG, msg);
    return MKID_OK;
}

// K7 on stream s for the sub-chunk's phase rows in d_raw: matched filter, baseline, trigger state
// machine (speculative segments + fix-up) into segments seg_off.. of the call's slot table, then
// the raw-phase history roll. Compaction (K8) runs once per call (compact_call).
static int run_trigger(mkid_ctx* c, const int16_t* raw, const SubPlan& sp, int32_t stride, int32_t seg_off,
                       int32_t capseg, hipStream_t s, bool roll = true) {
    const int C = c->C;
    KTime kt;
    TrigSpecArgs ta{raw,        c->d_rhist, c->d_fir,   c->d_thr,      c->d_rearm,   c->d_tstate,  c->d_tstate,
                    c->d_sspec, c->d_send,  c->d_slots, c->d_chcounts, c->d_scratch, c->d_reruns,
                    sp.J,       c->j0,      C,          sp.nseg,       sp.L,         sp.W,
                    capseg,     c->mode,    c->alpha,   c->kf,         c->kq,        c->base_thr,
                    c->cfg.dead_time, stride, seg_off, c->d_filt, c->d_refix, c->d_refix_pk};
    tstart(c, MKID_K_TRIGGER, &kt, s);
    HIPCHK(c, launch_trigger(ta, s));
    tstop(c, &kt, s);
    // the rolled history goes to the spare buffer and the two swap roles (enqueued kernels keep
    // the pointers they were launched with): no device-to-device copy per call. roll = false:
    // the caller rolls it together with the ADC history (raw_roll_job)
    if (roll) {
        HIPCHK(c, launch_hist_roll(c->d_rtmp, c->d_rhist, raw, kRawHist, sp.J, (int64_t)C * 2, s));
        std::swap(c->d_rhist, c->d_rtmp);
    }
    return MKID_OK;
}

// K8: one compaction over the call's [C][stride] slot table -> channel-major, time-ascending.
// Up to two history rolls ride along as extra blocks of the gather launch.
static int compact_call(mkid_ctx* c, int32_t stride, int32_t capseg, uint64_t* d_events, int64_t cap,
                        int64_t* d_counts, hipStream_t s, const RollJob* roll1 = nullptr,
                        const RollJob* roll2 = nullptr) {
    KTime kt;
    tstart(c, MKID_K_COMPACT, &kt, s);
    HIPCHK(c, launch_compact(c->d_slots, c->d_chcounts, (int64_t)c->C * stride, capseg, d_events, cap, d_counts,
                             c->d_scan, roll1, roll2, s));
    tstop(c, &kt, s);
    return MKID_OK;
}

// Fused front end: one front-end launch per sub-chunk (ADC -> phase, raw), then K7, one
// compaction per call, all on the context stream. (Round 2 also had an opt-in two-stream pipeline
// running a register-lean trigger beside the front end; it never paid — the front ends keep their
// SIMDs ~77 % VALU-busy, and the lean kernel alone is no faster than k_trig_spec — and was removed
// in round 3: profiles/r02/r02_v7_kbench_pipeline.json, r03_h_kbench_trig_lean_standalone*.json.)
static int process_fused(mkid_ctx* c, const int16_t* d_iq, int64_t n, float* d_phase, uint64_t* d_events,
                         int64_t cap, int64_t* d_counts) {
    const int C = c->C, N = c->N, M = c->M;
    const int64_t G = c->G;
    hipStream_t A = c->stream;
    std::vector<SubPlan> subs;
    int32_t stride = 0, capseg = 0;
    {
        int r = plan_call(c, n, subs, stride, capseg);
        if (r) return r;
    }
    // planned: from the first launch on the context carries an ADC stream, even if a later step of
    // this call fails (a failed planning / argument check leaves the stream kind as it was)
    c->stream_kind = 1;
    const uint32_t* x = (const uint32_t*)d_iq;
    c->last_J = 0;
    int32_t seg_off = 0;
    size_t si = 0;
    RollJob last_roll{};
    const Centring cen{c->d_ncen, c->d_cor, tap_offset(c)};
    for (int64_t off = 0; off < n; off += G, ++si) {
        const int64_t S = std::min<int64_t>(G, n - off);
        const int64_t K = S / M, J = S / N;
        int16_t* raw = c->d_raw + (off / N) * C;
        KTime kt;
        FrontArgs fa{};
        fa.x = x + off;
        fa.xhist = c->d_xhist;
        fa.pfbq = c->d_pfbq;
        fa.bins = c->d_bins;
        fa.lo = c->d_lo;
        fa.cen = cen;
        fa.phase = d_phase ? d_phase + (off / N) * C : nullptr;
        fa.raw = raw;
        fa.ysum = c->acc_on ? c->d_ysum : nullptr;
        fa.K = K;
        fa.k0 = c->k0;
        fa.avail = off;
        fa.P = c->P;
        fa.ncu = c->ncu;
        fa.taps = c->lpf;
        fa.iqtap = c->iq_ch >= 0 ? c->d_iqtap + (off / N) * 2 : nullptr;
        fa.iq_ch = c->iq_ch;
        fa.slot_ch = c->N == 2048 ? c->d_slot_ch : nullptr;   // k_front3 at N = 2048 only
        tstart(c, MKID_K_FRONT, &kt, A);
        HIPCHK(c, launch_fused(N, fa, A));
        tstop(c, &kt, A);
        if (c->fault_launch > 0 && ++c->launch_count == c->fault_launch)
            FAIL(c, MKID_E_HIP, "injected launch failure (MKID_FAULT_LAUNCH)");
        const bool last = off + S >= n;
        int r = run_trigger(c, raw, subs[si], stride, seg_off, capseg, A, !last);
        if (r) return r;
        if (last) {
            last_roll = RollJob{c->d_rtmp, c->d_rhist, raw, kRawHist, subs[si].J, (int64_t)C * 2};
        }
        seg_off += subs[si].nseg;
        c->k0 += K;
        c->j0 += J;
        c->last_J += J;
        c->last_subJ = J;
        c->last_raw_row = off / N;
    }
    {   // with the last sub-chunk's raw-phase history and the call's ADC history rolled in the
        // compaction's gather launch (no kernel of the call reads the rolled-to buffers)
        const RollJob xroll{c->d_xtmp, c->d_xhist, x, c->H, n, 4};
        int r = compact_call(c, stride, capseg, d_events, cap, d_counts, A, &last_roll, &xroll);
        if (r) return r;
    }
    std::swap(c->d_rhist, c->d_rtmp);
    std::swap(c->d_xhist, c->d_xtmp);
    c->iq_rows = c->iq_ch >= 0 ? n / N : 0;
    return MKID_OK;
}

// Split front end (channeliser on stream A, low-pass / trigger / compaction on stream B).
static int process_split(mkid_ctx* c, const int16_t* d_iq, int64_t n, float* d_phase, uint64_t* d_events,
                         int64_t cap, int64_t* d_counts) {
    const int C = c->C, N = c->N, M = c->M;
    const int64_t H = c->H;
    hipStream_t A = c->stream, B = c->sB;
    std::vector<SubPlan> subs;
    int32_t stride = 0, capseg = 0;
    {
        int r = plan_call(c, n, subs, stride, capseg);
        if (r) return r;
    }
    c->stream_kind = 1;   // planned (as process_fused)
    // B joins A's order (inputs written by earlier work on A, previous calls) ...
    HIPCHK(c, hipEventRecord(c->ev_start, A));
    HIPCHK(c, hipStreamWaitEvent(B, c->ev_start, 0));
    const uint32_t* x = (const uint32_t*)d_iq;
    const Centring cen{c->d_ncen, c->d_cor, tap_offset(c)};
    c->last_J = 0;
    int32_t seg_off = 0;
    size_t si = 0;
    const float2* zprev = c->d_zhist;  // the 24 frames before the current sub-chunk
    for (int64_t off = 0; off < n; off += c->G, ++si) {
        const int64_t S = std::min<int64_t>(c->G, n - off);
        const int64_t K = S / M, J = S / N;
        const int b = c->zi;
        float2* z = c->d_zb[b];
        KTime kt;
        // ---- stream A: channeliser into z[b] once its last reader is done ----
        HIPCHK(c, hipStreamWaitEvent(A, c->ev_zfree[b], 0));
        ChanArgs ca{x + off, c->d_xhist, c->d_pfb, c->d_bins, c->d_lo, z, K, c->k0, c->P, 0, 0, off};
        tstart(c, MKID_K_CHANNELIZE, &kt, A);
        HIPCHK(c, launch_channelize(N, ca, A));
        tstop(c, &kt, A);
        HIPCHK(c, hipEventRecord(c->ev_zready[b], A));

        // ---- stream B: low-pass + phase and trigger of this sub-chunk ----
        HIPCHK(c, hipStreamWaitEvent(B, c->ev_zready[b], 0));
        LpfArgs la{z, zprev, cen, d_phase ? d_phase + (off / N) * C : nullptr,
                   c->d_raw, c->acc_on ? c->d_ysum : nullptr, J, C, c->lpf,
                   c->iq_ch >= 0 ? c->d_iqtap + (off / N) * 2 : nullptr, c->iq_ch};
        tstart(c, MKID_K_FIR_PHASE, &kt, B);
        HIPCHK(c, launch_lpf_phase(la, B));
        tstop(c, &kt, B);
        if (off + S >= n || K < kLpfHist) {
            // carry the trailing 24 frames through d_zhist: always at the end of a call (next
            // call's history), and between sub-chunks too short to hold them
            HIPCHK(c, launch_hist_roll(c->d_ztmp, zprev, z, kLpfHist, K, (int64_t)C * 8, B));
            std::swap(c->d_zhist, c->d_ztmp);
            zprev = c->d_zhist;
            HIPCHK(c, hipEventRecord(c->ev_zfree[b], B));
        } else {
            zprev = z + (K - kLpfHist) * C;  // read in place by the next sub-chunk's low-pass
        }
        // the previous sub-chunk's buffer (history of the low-pass above) may now be overwritten
        HIPCHK(c, hipEventRecord(c->ev_zfree[b ^ 1], B));
        c->zi ^= 1;

        {
            int r = run_trigger(c, c->d_raw, subs[si], stride, seg_off, capseg, B);
            if (r) return r;
        }
        seg_off += subs[si].nseg;
        c->k0 += K;
        c->j0 += J;
        c->last_J += J;
        c->last_subJ = J;
        c->last_raw_row = 0;
    }
    {
        int r = compact_call(c, stride, capseg, d_events, cap, d_counts, B);
        if (r) return r;
    }
    // ADC history for the next call (all readers of d_xhist are channeliser launches on A)
    HIPCHK(c, launch_hist_roll(c->d_xtmp, c->d_xhist, x, H, n, 4, A));
    std::swap(c->d_xhist, c->d_xtmp);
    // ... and A (the caller's stream) waits for everything B did
    HIPCHK(c, hipEventRecord(c->ev_done, B));
    HIPCHK(c, hipStreamWaitEvent(A, c->ev_done, 0));
    c->iq_rows = c->iq_ch >= 0 ? n / N : 0;
    return MKID_OK;
}

int mkid_process_device(mkid_ctx* c, const int16_t* d_iq, int64_t n, float* d_phase, uint64_t* d_events,
                        int64_t cap, int64_t* d_counts) {
    if (!c || !d_iq || !d_counts || (cap > 0 && !d_events)) return MKID_E_ARG;
    if (n <= 0 || n % c->N != 0) FAIL(c, MKID_E_ARG, "nsamples must be a positive multiple of N");
    // the workspace (raw rows, IQ tap, slot table) is sized for max_chunk samples per call
    if (n > c->cfg.max_chunk) FAIL(c, MKID_E_ARG, "nsamples exceeds cfg.max_chunk");
    if (((uintptr_t)d_iq & 15) != 0) FAIL(c, MKID_E_ARG, "d_iq must be 16-byte aligned");
    if (c->stream_kind == 2)
        FAIL(c, MKID_E_STATE, "the context carries a phase-row stream (mkid_trigger_phase); mkid_reset_stream first");
    HIPCHK(c, hipSetDevice(c->device));
    const int r = c->fused ? process_fused(c, d_iq, n, d_phase, d_events, cap, d_counts)
                           : process_split(c, d_iq, n, d_phase, d_events, cap, d_counts);
    if (r == MKID_OK) acc_account(c, n / c->N);
    else if (c->acc_on) c->acc_rows = -1;   // some front-end launches may have added to the sums
    return r;
}

int mkid_trigger_phase(mkid_ctx* c, const int16_t* d_raw, int64_t rows, uint64_t* d_events, int64_t cap,
                       int64_t* d_counts) {
    if (!c || !d_raw || !d_counts || (cap > 0 && !d_events)) return MKID_E_ARG;
    if (rows <= 0 || rows > c->cfg.max_chunk / c->N) FAIL(c, MKID_E_ARG, "rows must be in 1 .. max_chunk/N");
    if (((uintptr_t)d_raw & 3) != 0) FAIL(c, MKID_E_ARG, "d_raw must be 4-byte aligned");
    if (c->stream_kind == 1)
        FAIL(c, MKID_E_STATE, "the context carries an ADC stream (mkid_process); mkid_reset_stream first");
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t s = c->stream;
    std::vector<SubPlan> subs;
    int32_t stride = 0, capseg = 0;
    {
        int r = plan_call(c, rows * c->N, subs, stride, capseg);
        if (r) return r;
    }
    c->stream_kind = 2;   // planned: the context now carries a phase-row stream (as process_fused)
    int32_t seg_off = 0;
    int64_t r0 = 0;
    for (const SubPlan& sp : subs) {
        int r = run_trigger(c, d_raw + r0 * c->C, sp, stride, seg_off, capseg, s);
        if (r) return r;
        seg_off += sp.nseg;
        r0 += sp.J;
        c->j0 += sp.J;
    }
    return compact_call(c, stride, capseg, d_events, cap, d_counts, s);
}

int mkid_process(mkid_ctx* c, const int16_t* iq, int64_t n, float* phase_out, uint64_t* events_out, int64_t cap,
                 int64_t* nevents) {
    if (!c || !iq || !nevents || (cap > 0 && !events_out)) return MKID_E_ARG;
    if (n <= 0 || n % c->N != 0) FAIL(c, MKID_E_ARG, "nsamples must be a positive multiple of N");
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t chunk = c->cfg.max_chunk;
    // hard bound for a whole call of `chunk` samples (per channel: J/(dead+3)+2 packets)
    const int64_t evcap = (int64_t)c->C * ((chunk / c->N) / (c->cfg.dead_time + 3) + 2);
    if (!c->d_in) {
        HIPCHK(c, dalloc(&c->d_in, (size_t)chunk));
        HIPCHK(c, dalloc(&c->d_phase_ws, (size_t)(chunk / c->N) * c->C));
        HIPCHK(c, dalloc(&c->d_ev_ws, (size_t)evcap));
    }
    int64_t produced = 0, written = 0;
    for (int64_t off = 0; off < n; off += chunk) {
        const int64_t S = std::min(chunk, n - off);
        HIPCHK(c, hipMemcpyAsync(c->d_in, iq + 2 * off, (size_t)S * 4, hipMemcpyHostToDevice, c->stream));
        int r = mkid_process_device(c, (const int16_t*)c->d_in, S, phase_out ? c->d_phase_ws : nullptr,
                                    c->d_ev_ws, evcap, c->d_counts);
        if (r) return r;
        int64_t cnt[2];
        HIPCHK(c, hipMemcpyAsync(cnt, c->d_counts, 16, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (phase_out)
            HIPCHK(c, hipMemcpyAsync(phase_out + (off / c->N) * c->C, c->d_phase_ws,
                                     (size_t)(S / c->N) * c->C * 4, hipMemcpyDeviceToHost, c->stream));
        const int64_t take = std::max<int64_t>(0, std::min(cnt[1], cap - written));
        if (take > 0)
            HIPCHK(c, hipMemcpyAsync(events_out + written, c->d_ev_ws, (size_t)take * 8, hipMemcpyDeviceToHost,
                                     c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        produced += cnt[0];
        written += take;
    }
    *nevents = produced;
    if (n > chunk) plan::merge_channel_major(events_out, written);   // chunks were compacted separately
    if (produced > written) FAIL(c, MKID_E_OVERFLOW, "event capacity exceeded; events dropped");
    return MKID_OK;
}

int mkid_last_raw_phase(mkid_ctx* c, const int16_t** d_raw, int64_t* nrows) {
    if (!c || !d_raw || !nrows) return MKID_E_ARG;
    *d_raw = c->d_raw + c->last_raw_row * c->C;
    *nrows = std::min(c->last_subJ, c->Jmax);
    return MKID_OK;
}

int mkid_read_raw_phase(mkid_ctx* c, int16_t* host_out, int64_t cap_rows, int64_t* rows) {
    if (!c || !rows || (cap_rows > 0 && !host_out)) return MKID_E_ARG;
    const int64_t avail = std::min(c->last_subJ, c->Jmax);
    *rows = avail;
    const int64_t n = std::min(avail, cap_rows);
    if (n <= 0) return MKID_OK;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(host_out, c->d_raw + c->last_raw_row * c->C, (size_t)n * c->C * 2,
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return MKID_OK;
}

int mkid_set_iq_tap(mkid_ctx* c, int32_t channel) {
    if (!c) return MKID_E_ARG;
    if (channel >= c->C) FAIL(c, MKID_E_ARG, "iq tap channel out of range");
    c->iq_ch = channel < 0 ? -1 : channel;
    c->iq_rows = 0;
    return MKID_OK;
}

int mkid_read_iq_tap(mkid_ctx* c, int16_t* host_iq, int64_t cap_rows, int64_t* rows) {
    if (!c || !rows || (cap_rows > 0 && !host_iq)) return MKID_E_ARG;
    *rows = c->iq_rows;
    const int64_t n = std::min(c->iq_rows, cap_rows);
    if (n <= 0) return MKID_OK;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(host_iq, c->d_iqtap, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return MKID_OK;
}

int mkid_trigger_reruns(mkid_ctx* c, int64_t* total) {
    if (!c || !total) return MKID_E_ARG;
    std::vector<int32_t> r(c->C);
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(r.data(), c->d_reruns, (size_t)c->C * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    int64_t s = 0;
    for (int v : r) s += v;
    *total = s;
    return MKID_OK;
}

int mkid_set_accumulator(mkid_ctx* c, int32_t enable) {
    if (!c) return MKID_E_ARG;
    if (enable != 0 && enable != 1) FAIL(c, MKID_E_ARG, "enable must be 0 or 1");
    if (enable) {   // every arm starts a new average (avgIQ_ctrl strobe + startAccumulator 1)
        HIPCHK(c, hipSetDevice(c->device));
        HIPCHK(c, hipMemsetAsync(c->d_ysum, 0, (size_t)c->C * 16, c->stream));
        c->acc_rows = 0;
        std::fill(c->acc_off.begin(), c->acc_off.end(), 0.0);
    }
    c->acc_on = enable != 0;
    return MKID_OK;
}

int mkid_avg_iq(mkid_ctx* c, float* mi, float* mq) {
    if (!c || !mi || !mq) return MKID_E_ARG;
    if (c->acc_rows < 0)
        FAIL(c, MKID_E_STATE, "a process call failed while the avgIQ accumulator was armed: re-arm it");
    if (c->acc_rows == 0)
        FAIL(c, MKID_E_STATE, "the avgIQ accumulator holds no rows: arm it (mkid_set_accumulator) before processing");
    std::vector<long long> s(2 * (size_t)c->C);
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(s.data(), c->d_ysum, (size_t)c->C * 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const double inv = 1.0 / (double)c->acc_rows, scale = 1.0 / (double)(1 << kYsumFrac);
    for (int i = 0; i < c->C; ++i) {
        mi[i] = (float)(((double)s[2 * i] * scale + c->acc_off[2 * i]) * inv);
        mq[i] = (float)(((double)s[2 * i + 1] * scale + c->acc_off[2 * i + 1]) * inv);
    }
    return MKID_OK;
}

int mkid_replay_trigger(mkid_ctx* c, const int16_t* d_raw, int64_t n, int64_t ld, int32_t nch,
                        const mkid_replay_cfg* rc, int32_t* d_hits, int32_t cap, int32_t* d_counts) {
    if (!c || !d_raw || !rc || !d_counts || (cap > 0 && !d_hits)) return MKID_E_ARG;
    if (n <= 0 || nch <= 0 || ld < nch || cap < 0) FAIL(c, MKID_E_ARG, "replay: bad shape");
    if (rc->mode != MKID_REPLAY_ROLLING && rc->mode != MKID_REPLAY_BLOCK) FAIL(c, MKID_E_ARG, "replay: bad mode");
    if (rc->length <= 0 || rc->start < 0 || rc->need < 0 || rc->skip <= 0)
        FAIL(c, MKID_E_ARG, "replay: length/start/need/skip out of range");
    if (rc->mode == MKID_REPLAY_ROLLING && rc->start < rc->length)
        FAIL(c, MKID_E_ARG, "replay: rolling start must be >= meanlength");
    HIPCHK(c, hipSetDevice(c->device));
    const size_t nf = (size_t)nch * (size_t)((n + 31) / 32);
    const size_t nm = rc->mode == MKID_REPLAY_BLOCK ? (size_t)nch * (size_t)(n / rc->length) : 0;
    if (nf > c->rflags_n) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (c->d_rflags) HIPCHK(c, hipFree(c->d_rflags));
        c->d_rflags = nullptr;
        c->rflags_n = 0;
        HIPCHK(c, dalloc(&c->d_rflags, nf));
        c->rflags_n = nf;
    }
    if (nm > c->rmeans_n) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (c->d_rmeans) HIPCHK(c, hipFree(c->d_rmeans));
        c->d_rmeans = nullptr;
        c->rmeans_n = 0;
        HIPCHK(c, dalloc(&c->d_rmeans, nm));
        c->rmeans_n = nm;
    }
    HIPCHK(c, launch_replay(d_raw, n, ld, nch, rc->mode, rc->length, rc->start, rc->need, rc->skip,
                            rc->wrap_negative, rc->threshold_deg, c->d_rflags, c->d_rmeans, d_hits, cap,
                            d_counts, c->stream));
    return MKID_OK;
}

int mkid_make_template(mkid_ctx* c, const float* d_I, const float* d_Q, int64_t P, double* d_template,
                       double* d_noise, mkid_template_info* info) {
    if (!c || !d_I || !d_Q || !d_template || !d_noise || !info) return MKID_E_ARG;
    if (P <= 0) FAIL(c, MKID_E_ARG, "make_template: need pulses");
    HIPCHK(c, hipSetDevice(c->device));
    const size_t N = 2000, NN = 800;
    DevBufs b;
    float *I, *Q, *refmed;
    double *rows, *nrows, *peaks, *scratch, *tP, *stats;
    int32_t *accept, *appended;
    HIPCHK(c, b.get(&I, (size_t)P * N));
    HIPCHK(c, b.get(&Q, (size_t)P * N));
    HIPCHK(c, b.get(&rows, (size_t)P * N));
    HIPCHK(c, b.get(&nrows, (size_t)P * NN));
    HIPCHK(c, b.get(&peaks, (size_t)P));
    HIPCHK(c, b.get(&scratch, (size_t)2 * P + 8));
    HIPCHK(c, b.get(&tP, N));
    HIPCHK(c, b.get(&stats, 8));
    HIPCHK(c, b.get(&refmed, 2));
    HIPCHK(c, b.get(&accept, (size_t)P));
    HIPCHK(c, b.get(&appended, (size_t)P));
    hipStream_t s = c->stream;
    HIPCHK(c, hipMemcpyAsync(I, d_I, (size_t)P * N * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(c, hipMemcpyAsync(Q, d_Q, (size_t)P * N * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(c, hipMemsetAsync(appended, 0, (size_t)P * 4, s));
    HIPCHK(c, hipMemsetAsync(stats, 0, 64, s));
    hipError_t e = launch_make_template(I, Q, P, rows, nrows, accept, peaks, appended, scratch, tP, d_template,
                                        d_noise, stats, refmed, s);
    if (e == hipErrorInvalidValue) FAIL(c, MKID_E_STATE, "make_template: no pulse passed the first pass");
    HIPCHK(c, e);
    double st[5];
    std::vector<double> t(N);
    HIPCHK(c, hipMemcpyAsync(st, stats, 40, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(t.data(), d_template, N * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    info->pm = st[0];
    info->pdev = st[1];
    info->count1 = st[3];
    info->count = st[4];
    info->flag = (st[4] < 500 || st[0] < 10 || st[0] > 150) ? 1 : 0;
    int ps = 0;
    for (size_t i = 1; i < N; ++i)
        if (t[i] > t[ps]) ps = (int)i;
    info->pstart = ps;
    return MKID_OK;
}

int mkid_optimal_filter(mkid_ctx* c, const double* d_template, const double* d_noise, int32_t pre, int32_t ncoeff,
                        double* d_coeff) {
    if (!c || !d_template || !d_noise || !d_coeff) return MKID_E_ARG;
    if (pre < 10 || pre > 2000 || ncoeff <= 0 || ncoeff > 800) FAIL(c, MKID_E_ARG, "optimal_filter: bad pre/ncoeff");
    HIPCHK(c, hipSetDevice(c->device));
    DevBufs b;
    double* work;
    HIPCHK(c, b.get(&work, 3 * 800));
    HIPCHK(c, launch_optimal_filter(d_template, d_noise, pre, ncoeff, d_coeff, work, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return MKID_OK;
}

int mkid_set_pulse_filter(mkid_ctx* c, const float* coeff, int32_t nch, int32_t ncoeff, int32_t pre) {
    if (!c || !coeff) return MKID_E_ARG;
    if (nch != c->C) FAIL(c, MKID_E_ARG, "pulse filter: need one filter per channel");
    if (ncoeff < 1 || ncoeff > 4096 || pre < 0) FAIL(c, MKID_E_ARG, "pulse filter: bad ncoeff/pre");
    HIPCHK(c, hipSetDevice(c->device));
    if (c->d_hcoeff) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipFree(c->d_hcoeff));
        c->d_hcoeff = nullptr;
    }
    HIPCHK(c, dalloc(&c->d_hcoeff, (size_t)nch * ncoeff));
    if (c->d_phist) {
        HIPCHK(c, hipFree(c->d_phist));
        HIPCHK(c, hipFree(c->d_phist_tmp));
        c->d_phist = c->d_phist_tmp = nullptr;
    }
    HIPCHK(c, dalloc(&c->d_phist, (size_t)nch * ncoeff));
    HIPCHK(c, dalloc(&c->d_phist_tmp, (size_t)nch * ncoeff));
    c->phist_end = -1;
    c->phist_rows = 0;
    c->h_ncoeff = ncoeff;
    c->h_pre = pre;
    return upload(c, c->d_hcoeff, coeff, (size_t)nch * ncoeff * 4);
}

static int pulse_heights(mkid_ctx* c, const float* d_phase, int64_t rows, int64_t j0, const uint64_t* d_events,
                         const int64_t* d_n, int64_t n, float* d_heights) {
    if (!c || (n > 0 && (!d_phase || !d_events || !d_heights))) return MKID_E_ARG;
    if (rows < 0 || j0 < 0 || n < 0) FAIL(c, MKID_E_ARG, "pulse heights: negative rows/j0/n");
    if (!c->d_hcoeff) FAIL(c, MKID_E_STATE, "pulse heights: no filter set (mkid_set_pulse_filter)");
    HIPCHK(c, hipSetDevice(c->device));
    // the carried rows precede this call's rows only if the calls are contiguous in j
    const int64_t hrows = (c->phist_end == j0) ? c->phist_rows : 0;
    const int64_t H = c->h_ncoeff;   // d_phist: H rows, the valid ones are its last phist_rows
    HeightArgs a{d_phase, d_events, c->d_hcoeff, d_heights, rows, j0, n, c->C, c->h_ncoeff, c->h_pre, d_n,
                 c->d_phist + (H - hrows) * c->C, hrows, c->ncu, 0};
    KTime kt;
    tstart(c, MKID_K_HEIGHTS, &kt, c->stream);
    HIPCHK(c, launch_pulse_heights(a, c->stream));
    tstop(c, &kt, c->stream);
    // keep the last H rows of (history, these rows) for the next call's early windows
    if (rows > 0) {
        HIPCHK(c, launch_hist_roll(c->d_phist_tmp, c->d_phist, d_phase, H, rows, (int64_t)c->C * 4, c->stream));
        std::swap(c->d_phist, c->d_phist_tmp);
        c->phist_rows = std::min<int64_t>(H, hrows + rows);
        c->phist_end = j0 + rows;
    }
    return MKID_OK;
}

int mkid_pulse_heights(mkid_ctx* c, const float* d_phase, int64_t rows, int64_t j0, const uint64_t* d_events,
                       int64_t n, float* d_heights) {
    return pulse_heights(c, d_phase, rows, j0, d_events, nullptr, n, d_heights);
}

int mkid_pulse_heights_counted(mkid_ctx* c, const float* d_phase, int64_t rows, int64_t j0,
                               const uint64_t* d_events, const int64_t* d_count, int64_t cap, float* d_heights) {
    if (!d_count) return MKID_E_ARG;
    return pulse_heights(c, d_phase, rows, j0, d_events, d_count, cap, d_heights);
}

int mkid_stream_copy(mkid_ctx* c, void* d_dst, const void* d_src, int64_t bytes) {
    if (!c || !d_dst || !d_src || bytes < 0) return MKID_E_ARG;
    if (bytes % 16 != 0 || ((uintptr_t)d_dst & 15) != 0 || ((uintptr_t)d_src & 15) != 0)
        FAIL(c, MKID_E_ARG, "stream copy: 16-byte aligned pointers and sizes only");
    HIPCHK(c, hipSetDevice(c->device));
    KTime kt;
    tstart(c, MKID_K_COPY, &kt, c->stream);
    HIPCHK(c, launch_stream_copy(d_dst, d_src, bytes, c->stream));
    tstop(c, &kt, c->stream);
    return MKID_OK;
}

int mkid_set_timing_mask(mkid_ctx* c, uint32_t mask) {
    if (!c) return MKID_E_ARG;
    if ((mask & ~((1u << MKID_K_COUNT) - 1u)) != 0) FAIL(c, MKID_E_ARG, "timing mask: an OR of MKID_TIMING_ONLY(k)");
    int r = flush_timing(c);
    if (r) return r;
    c->timing = mask != 0;
    c->timing_mask = mask;
    for (int k = 0; k < MKID_K_COUNT; ++k) { c->tot_ms[k] = 0; c->launches[k] = 0; }
    return MKID_OK;
}

int mkid_set_timing(mkid_ctx* c, int32_t enable) {
    return mkid_set_timing_mask(c, enable != 0 ? (1u << MKID_K_COUNT) - 1u : 0u);
}

int mkid_get_timing(mkid_ctx* c, int32_t k, double* total_ms, int64_t* launches) {
    if (!c || k < 0 || k >= MKID_K_COUNT || !total_ms || !launches) return MKID_E_ARG;
    int r = flush_timing(c);
    if (r) return r;
    *total_ms = c->tot_ms[k];
    *launches = c->launches[k];
    return MKID_OK;
}

const char* mkid_kernel_name(int32_t k) {
    static const char* names[MKID_K_COUNT] = {"k_channelize", "k_lpf_phase", "k_trigger", "k_compact",
                                              "k_front",      "k_stream_copy", "k_pulse_heights"};
    return (k >= 0 && k < MKID_K_COUNT) ? names[k] : "?";
}

int mkid_synth_adc(mkid_ctx* c, int16_t* d_out, int64_t n, int64_t n0, const int16_t* d_base,
                   const mkid_synth_tone* d_tones, const mkid_pulse* d_pulses, int64_t npulses, float tr,
                   float tf, int32_t window, float sigma, uint32_t seed) {
    if (!c || !d_out || !d_base || n < 0 || (npulses > 0 && (!d_pulses || !d_tones))) return MKID_E_ARG;
    if (tr <= 0.f || tf <= 0.f || window < 0) FAIL(c, MKID_E_ARG, "bad pulse shape");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, launch_synth(d_out, n, n0, d_base, d_tones, d_pulses, npulses, tr, tf, window, sigma, seed,
                           c->stream));
    return MKID_OK;
}

int mkid_pack_reference(const uint64_t* wide, int64_t n, uint64_t* out) {
    if ((!wide || !out) && n > 0) return MKID_E_ARG;
    return plan::pack_reference(wide, n, out) == 0 ? MKID_OK : MKID_E_ARG;
}

}  // extern "C"
