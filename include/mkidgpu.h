/*
 * mkidgpu.h — flat C ABI of the MI355X MKID channeliser + phase/pulse-trigger hot path.
 *
 * This library replaces the ROACH FPGA firmware that creanero/MKIDS_SDR configures over katcp
 * (the firmware itself is absent from the reference: .MISSING_LARGE_BLOBS:1-27). Each entry point
 * below replaces one group of register/BRAM accesses the reference's host code makes; the
 * reference call site is cited on every declaration (paths relative to the reference root).
 *
 * ABI rules
 *   - every entry point returns int: 0 = ok, negative = MKID_E_* ; mkid_last_error() gives text.
 *   - no C++ exception crosses the ABI; buffers are caller-owned; plain pointers and sizes only.
 *   - one HIP stream per context (its own, or one handed in by mkid_set_stream); a context is not
 *     thread-safe; distinct contexts (one per GPU / feedline) may run concurrently.
 *   - *_device entry points take device pointers and are fully asynchronous on the context's
 *     stream (graph-capturable); the host-pointer entry points copy in/out and synchronise.
 *
 * Geometry: C channels, N = 2C point FFT, hop M = N/2 (2x oversampled), T PFB taps per branch.
 * Input: int16 I/Q pairs (interleaved, I first) at fs. Output: per-channel phase at fs/N
 * (layout [J][C], time-major, J = nsamples/N) and 64-bit photon packets (see MKID_PKT_*).
 */
#ifndef MKIDGPU_H
#define MKIDGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MKID_OK 0
#define MKID_E_ARG (-1)       /* bad argument / shape mismatch                      */
#define MKID_E_HIP (-2)       /* HIP runtime failure (message in mkid_last_error)   */
#define MKID_E_STATE (-3)     /* call order violated (e.g. process before config)    */
#define MKID_E_OVERFLOW (-4)  /* event capacity exceeded; events were dropped         */
#define MKID_E_NODEV (-5)     /* no HIP device                                       */

/* Baseline modes of the trigger (K7). The reference writes these registers:
 *   capture_Baseline_alpha  (DataReadout/ChannelizerControls/lib/set_alpha.py:10-17, Fix12_9)
 *   capture_base_Kf/Kq      (lib/set_svf.py:29-35, Fix18_16)
 *   capture_base_thresh     (lib/set_base_thresh.py:9-17, Fix16_13; B_BASE_THRESH setEnvironment.sh:26) */
#define MKID_BASE_NONE 0
#define MKID_BASE_EMA 1
#define MKID_BASE_SVF 2

/* Wide 64-bit photon packet emitted by the device (channel field widened for C > 255):
 *   [63:52] channel (12b) | [51:40] peak Fix12_9 offset (x/2^9-4 rad) | [39:28] baseline Fix12_9
 *   offset | [27:0] phase-sample index mod 2^28.
 * The reference 64-bit packet (ch 8b | peak 12b | p1 12b | base 12b | ts 20b,
 * ROACH_Pulses.py:796-832, PacketMaster.c:291-292) is produced on the host by
 * mkid_pack_reference() for C <= 254. */
#define MKID_PKT_CH_SHIFT 52
#define MKID_PKT_PEAK_SHIFT 40
#define MKID_PKT_BASE_SHIFT 28
#define MKID_PKT_TS_MASK ((1ull << 28) - 1)

/* Front-end (K1-K6) execution: one fused kernel (z stays on-chip) or two kernels with the complex
 * baseband z staged in HBM. Results agree to float rounding; AUTO picks fused where supported. */
#define MKID_FRONT_AUTO 0
#define MKID_FRONT_SPLIT 1

typedef struct mkid_ctx mkid_ctx;

typedef struct mkid_cfg {
    int32_t n_channels;        /* C; ROACH_Setup.py:515 (256)                                  */
    int32_t fft_len;           /* N = 2C; ROACH_Setup.py:507 fft_len = 2**9                    */
    int32_t pfb_taps;          /* T taps per PFB branch (build decision, 4)                    */
    int32_t fir_taps;          /* 26; ROACH_Pulses.py:61                                      */
    int32_t dds_entries;       /* P = 2^16 / C LO samples per channel; ROACH_Setup.py:521-530 */
    int32_t dead_time;         /* trigger dead time in phase samples (build decision)         */
    int32_t max_events_per_ch; /* per-call event capacity per channel (0 = derive from chunk) */
    int32_t front;             /* MKID_FRONT_AUTO (fused K1-K6 kernel, N = 128..4096) or
                                  MKID_FRONT_SPLIT (channeliser + low-pass kernels, z in HBM)  */
    int64_t max_chunk;         /* largest nsamples per process call (workspace sizing)        */
    double sample_rate;        /* fs, complex S/s; ROACH_Setup.py:82                           */
} mkid_cfg;

/* Fill *cfg with defaults for C channels (N=2C, T=4, 26 taps, P=65536/C, fs=512e6). */
int mkid_default_cfg(mkid_cfg* cfg, int32_t n_channels);

/* Create a context on HIP device `device`. Replaces FpgaClient(ip,7147)+progdev(bof):
 * ROACH_Setup.py:112-115, ROACH_Pulses.py:51-52. */
int mkid_create(const mkid_cfg* cfg, int32_t device, mkid_ctx** out);
int mkid_destroy(mkid_ctx* ctx);
const char* mkid_last_error(const mkid_ctx* ctx);
/* Error text for failures that happen before a context exists (mkid_create). */
const char* mkid_global_error(void);
int mkid_get_cfg(const mkid_ctx* ctx, mkid_cfg* out);

/* Run the context's kernels on an external hipStream_t (e.g. torch's current stream). NULL
 * restores the context's own stream. */
int mkid_set_stream(mkid_ctx* ctx, void* hip_stream);

/* PFB prototype filter, T*N float coefficients (build decision: the firmware's taps are not in
 * the reference). Applied as 16-bit integers, like an FPGA PFB's fixed-point coefficients:
 * h_q = rint(h * 2^S) with the largest S such that every point's sum_tau |h_q[tau N + p]| <= 65535
 * and every |h_q| <= 32767; the effective taps are h_q * 2^-S (mkids_sdr_amd.pfb.effective_taps). */
int mkid_set_pfb(mkid_ctx* ctx, const float* coeffs, int32_t n);
/* Host-only (no device needed): the effective taps h_q * 2^-S of mkid_set_pfb and S. */
int mkid_pfb_effective_taps(const float* coeffs, int32_t T, int32_t N, float* out, int32_t* shift);
/* Host-only: the channel order the fused front ends give their select threads for a bin set:
 * out[slot] = channel. C = 1024 (k_front3, N = 2048): slot st + 512 q is read by thread st in
 * instruction q, and each select wave keeps its own 128 channels. C = 2048 (the k_front5 layout,
 * N = 4096): slot 64 sw + l + 512 q (select waves sw < 8, q < 3) or 1536 + 64 v + l + 256 q (v < 4,
 * q < 2), each wave keeping the natural channels of its slots; reported for tools/lds_assign.py,
 * not applied (it cut k_front5's LDS conflict cycles 2.6x but cost 2.5-6 % in time, DESIGN.md
 * §5.3). Within a wave the order puts each
 * half-wave's 32 Y reads on distinct LDS bank pairs where the bins allow. A permutation of 0..C-1
 * (the identity for C other than 1024 and 2048). Results do not depend on it: each channel's
 * arithmetic is unchanged. Exposed for tests and tools/lds_assign.py; MKID_SLOT_ORDER=0 at context
 * creation disables it. */
int mkid_slot_order(const int32_t* bins, int32_t C, int16_t* out);

/* Coarse FFT bin per channel: replaces write_int('bins'), write_int('load_bins',(i<<1)+1)
 * (ROACH_Setup.py:534-550; ROACH_Pulses.py:958-974). bins[c] in [0,N). */
int mkid_set_bins(mkid_ctx* ctx, const int32_t* bins, int32_t n);

/* Per-channel DDS LO LUT, de-interleaved and un-shifted: lut_i/lut_q are [C][P] int16, the
 * freqCombLUT('no',...) output of define_DDS_LUT (ROACH_Setup.py:506-532) before it is woven
 * into dram_memory (ROACH_Setup.py:552-570). The device mixes by conj(LUT)/2^15. */
int mkid_set_dds(mkid_ctx* ctx, const int16_t* lut_i, const int16_t* lut_q, int32_t entries_per_ch);

/* IQ low-pass (K5) taps, int12 Fix12_11 (int(lpf*(2**11-1)), ROACH_Pulses.py:69,88-92), shared
 * by all channels, applied to the DDC output with decimation by 2. */
int mkid_set_lpf(mkid_ctx* ctx, const int16_t* taps12, int32_t ntaps);

/* Per-channel matched-filter taps [C][26] int12: replaces FIR_b{2n}b{2n+1} + FIR_load_coeff
 * (ROACH_Pulses.py:59-111). All-zero taps delete a channel (no triggers). */
int mkid_set_fir(mkid_ctx* ctx, const int16_t* taps12, int32_t n_channels, int32_t ntaps);

/* IQ loop centres [C] in channel-output units: replaces conv_phase_centers /
 * conv_phase_load_centers (ROACH_Setup.py:595-605). phase = atan2(Q - qc, I - ic) is evaluated
 * with the centre subtracted inside the low-pass (sum_i g_i (z_i - c/G) + r, G = sum of the
 * low-pass taps, r the float64 residual of G c'), so the fp32 error of the phase does not grow
 * with |centre| / loop radius. Centres must be finite. */
int mkid_set_centers(mkid_ctx* ctx, const float* ic, const float* qc, int32_t n);

/* Per-channel trigger thresholds [C], Fix16_13 raw units relative to baseline (negative-going):
 * replaces capture_threshold / capture_load_thresh (ROACH_Pulses.py:211-354). */
int mkid_set_thresholds(mkid_ctx* ctx, const int32_t* thr, int32_t n);

/* Baseline: mode MKID_BASE_*, alpha Fix12_9 in 0..1024 (gain <= 2.0; larger gains diverge),
 * kf/kq Fix18_16, base_thr Fix16_13 (0 = no gate). */
int mkid_set_baseline(mkid_ctx* ctx, int32_t mode, int32_t alpha, int32_t kf, int32_t kq,
                      int32_t base_thr);

/* Trigger re-arm hysteresis (K7 state machine, build decision: the firmware is absent): after its
 * dead time a channel re-arms once e = f - baseline >= thr_c - floor(thr_c * frac_q8 / 256), i.e.
 * at a level moved from its threshold toward the baseline by frac_q8 / 256 (0..256). 0 (the
 * default) re-arms at the threshold, the round-1..4 rule, bit-identical. Without it a slow baseline
 * (SVF) lets the pulse tail re-cross the threshold after the dead time; the
 * reference's host replay holds off a fixed 1000 samples instead (pulse_triggering_v2.py:104-174).
 * Kept across mkid_set_thresholds (the levels follow the thresholds). */
int mkid_set_rearm(mkid_ctx* ctx, int32_t frac_q8);

/* Forget all stream state (PFB/FIR history, baselines, trigger state, sample counter). */
int mkid_reset_stream(mkid_ctx* ctx);

/* Process nsamples (multiple of N) I/Q pairs, host pointers, synchronous. phase_out (nullable)
 * receives [nsamples/N][C] float32 rad; events_out receives up to cap packets, channel-major and
 * time-ascending within a channel over the whole call (a call longer than cfg.max_chunk runs as
 * max_chunk pieces whose lists are merged on the host); *nevents = packets produced (> cap =>
 * MKID_E_OVERFLOW; the packets kept are then the first cap entries of the pieces' channel-major
 * lists concatenated in piece order: earlier pieces whole, the low channels of the piece that
 * overflows, nothing of later pieces; merged channel-major as above). */
int mkid_process(mkid_ctx* ctx, const int16_t* iq, int64_t nsamples, float* phase_out,
                 uint64_t* events_out, int64_t cap, int64_t* nevents);

/* Same with device pointers, asynchronous on the context stream; nsamples <= cfg.max_chunk (the
 * workspace size; MKID_E_ARG otherwise). d_counts is a device int64[2]: [0] = packets produced
 * (may exceed cap), [1] = packets written, channel-major and time-ascending within a channel over
 * the whole call. d_phase may be NULL (the phase stream is then not materialised; the trigger
 * still runs on the Fix16_13 phase). */
int mkid_process_device(mkid_ctx* ctx, const int16_t* d_iq, int64_t nsamples, float* d_phase,
                        uint64_t* d_events, int64_t cap, int64_t* d_counts /* [2] */);

/* K7 + K8 alone on caller-supplied Fix16_13 phase rows [rows][C] int16 (device pointer, e.g. a
 * snapshot uploaded by the caller: the reference runs its trigger on snapshots too,
 * ROACH_Pulses.py:211-354, 614-727): matched filter, baseline, trigger, packets, with the
 * context's carried trigger state and phase-sample counter (advanced by rows). rows <=
 * max_chunk/N. d_counts / packet order as mkid_process_device. Asynchronous on the context stream.
 * A context carries ONE stream: ADC samples (mkid_process*) or phase rows (this call). Calling one
 * kind after the other without mkid_reset_stream fails with MKID_E_STATE, so a snapshot never
 * advances the trigger state, the raw history or the packet stamps of a live ADC stream (use a
 * second context for snapshots taken beside a running feedline). */
int mkid_trigger_phase(mkid_ctx* ctx, const int16_t* d_raw, int64_t rows, uint64_t* d_events,
                       int64_t cap, int64_t* d_counts /* [2] */);

/* Fixed-point phase of the last processed call, [J][C] int16 Fix16_13 (the trigger's input),
 * device pointer valid until the next process call. Replaces the snapPhase_bram source
 * (ROACH_Pulses.py:357-378). */
int mkid_last_raw_phase(mkid_ctx* ctx, const int16_t** d_raw, int64_t* nrows);
/* Host copy of the same rows (at most cap_rows rows of C int16; *rows = rows available): the
 * snapshot readback (conv_phase_snapPhase_bram / qdr0 longsnapshot, ROACH_Pulses.py:433-551). */
int mkid_read_raw_phase(mkid_ctx* ctx, int16_t* host_out, int64_t cap_rows, int64_t* rows);

/* IQ snapshot tap (conv_phase_ch_we_IQ / conv_phase_snapIQ_bram, pulse_triggering_IQ.py:36,
 * 113-147): record the low-pass output y of one channel (channel < 0: off) for the rows of each
 * process call, as int16 I/Q pairs in ADC-count units (the units of mkid_avg_iq and the IQ
 * centres; saturated). mkid_read_iq_tap copies the last call's rows [rows][2] to the host. */
int mkid_set_iq_tap(mkid_ctx* ctx, int32_t channel);
int mkid_read_iq_tap(mkid_ctx* ctx, int16_t* host_iq, int64_t cap_rows, int64_t* rows);

/* Diagnostic: trigger segments of the last sub-chunk whose speculative start state had to be
 * re-run by the exact fix-up pass (0 = all speculation was right; results are exact either way). */
int mkid_trigger_reruns(mkid_ctx* ctx, int64_t* total);

/* avgIQ accumulator (K9): replaces startAccumulator / avgIQ_ctrl (ROACH_Setup.py:654-659,
 * rotateLoopsReady). enable = 1 arms it — the sums restart on every call with 1, armed or not
 * (the avgIQ_ctrl strobe the reference writes before each startAccumulator 1) — and every
 * following process call adds its rows; 0 stops it and keeps the sums. Off after mkid_create; the
 * front ends skip the accumulation while it is off. mkid_reset_stream clears the sums and keeps
 * the armed state. */
int mkid_set_accumulator(mkid_ctx* ctx, int32_t enable);
/* Per-channel mean I/Q (low-pass output y, ADC-count units) over the rows accumulated since the
 * accumulator was last armed (avgIQ_bram, ROACH_Setup.py:654-662), [C] each. MKID_E_STATE when it
 * holds no rows, or when a process call failed while it was armed (its sums may hold part of that
 * call; re-arm to start a new average). */
int mkid_avg_iq(mkid_ctx* ctx, float* mean_i, float* mean_q);

/* Re-encode wide device packets as the reference 64-bit packet (host memory, C <= 254):
 *   [63:56] ch | [55:44] peak | [43:32] p1 = peak-base+2048 | [31:20] base | [19:0] ts mod 2^20
 * (ROACH_Pulses.py:805-832 decode; PacketMaster.c:291-292 assembly; ch 255 = end-of-second). */
int mkid_pack_reference(const uint64_t* wide, int64_t n, uint64_t* out);

/* Host-replay triggers of the reference on device phase. Input: Fix16_13
 * phase int16 [n][ld] (e.g. mkid_last_raw_phase, or snapshots uploaded by the caller), columns
 * 0..nch-1 are channels. Phase in degrees = raw*360/2^16*4/pi (pulse_triggering_v2.py:93-95).
 *   MKID_REPLAY_ROLLING  pulse_triggering_v2.py:104-174: start = 100+m, need = skip = pulselength,
 *                        length = m (meanlength, 20), |mean(x[j-m:j]) - x[j]| > threshold
 *   MKID_REPLAY_BLOCK    pulse_triggering.py:109-208 (start 100, need 300, skip 200, wrap on) and
 *                        ROACH_Pulses.py:614-727 (start 500): length = averagelength (2^k),
 *                        |mean(block(j)) - x[j]| > threshold
 * Hits (sample indices) go to d_hits[c*cap + i], i < cap; d_counts[c] = hits found (may exceed
 * cap: then hits were dropped). Means use numpy's pairwise float64 summation order, so the hit
 * lists equal the reference's numpy loops exactly. Runs on the context stream. */
#define MKID_REPLAY_ROLLING 0
#define MKID_REPLAY_BLOCK 1
typedef struct mkid_replay_cfg {
    int32_t mode;          /* MKID_REPLAY_ROLLING / MKID_REPLAY_BLOCK                       */
    int32_t length;        /* rolling: meanlength m; block: averagelength A                 */
    int32_t start;         /* first index tested ("bob")                                    */
    int32_t need;          /* stop when bob + need > n                                      */
    int32_t skip;          /* advance after a hit                                           */
    int32_t wrap_negative; /* add 360 deg to negative phase first (pulse_triggering.py:110)  */
    double threshold_deg;  /* strict: |mean - x| > threshold                                */
} mkid_replay_cfg;
int mkid_replay_trigger(mkid_ctx* ctx, const int16_t* d_raw, int64_t n, int64_t ld, int32_t nch,
                        const mkid_replay_cfg* cfg, int32_t* d_hits, int32_t cap, int32_t* d_counts);

/* Pulse template and near-optimal filter: MakeTemplate
 * (DataReadout/ReadoutControls/lib/pulses.py:239-427) on device for one resonator's pulses, the
 * reference's RawPulse rows I, Q float32 [npulses][2000] (pulses.py:30-43; not modified).
 * Outputs the PulseAnalysis fields (pulses.py:44-51): template [2000] f64 (deg-normalised,
 * peak at pstart), noise PSD [800] f64, and the scalars below. Fails with MKID_E_STATE when no
 * pulse survives the first pass. */
typedef struct mkid_template_info {
    double count;   /* pulses in the final template (pass 2)                         */
    double count1;  /* pulses in the preliminary template (pass 1, first 1000 pulses) */
    double pm;      /* median of first-pass peaks > 15 deg (pulses.py:335)            */
    double pdev;    /* their std                                                      */
    int32_t flag;   /* 1 if count < 500 or pm < 10 or pm > 150 (pulses.py:409-412)    */
    int32_t pstart; /* index of the template maximum (pulses.py:415)                  */
} mkid_template_info;
int mkid_make_template(mkid_ctx* ctx, const float* d_I, const float* d_Q, int64_t npulses,
                       double* d_template, double* d_noise, mkid_template_info* info);
/* The optimal filter the reference stubs (pulses.py:398; PulseAnalysis.coeff Float32Col(100)):
 * correlation weights g = ifft(S / J) (S = fft of the 800-sample template window starting `pre`
 * samples before its peak, deg->rad; J = noise PSD; DC bin zeroed), normalised to unit response
 * to the template; d_coeff[0..ncoeff) = g[pre-10 ...]. Device in, device out. */
int mkid_optimal_filter(mkid_ctx* ctx, const double* d_template, const double* d_noise, int32_t pre,
                        int32_t ncoeff, double* d_coeff);

/* Per-packet optimal-filter pulse height, fp32 (BASELINE config 5): the filter above (or any
 * per-channel FIR) applied to the phase stream at each photon packet,
 *     h = sum_{i < ncoeff} coeff[ch][i] * phase[ts - pre + i][ch]     (phase in rad)
 * the estimate the reference's PulseAnalysis.coeff was meant for (pulses.py:44-51, 398).
 * mkid_set_pulse_filter: host coeff [nch = C][ncoeff] fp32, 1 <= ncoeff <= 4096, 0 <= pre.
 * mkid_pulse_heights: d_phase holds the device phase rows of global phase indices
 * j0 .. j0 + rows - 1 ([rows][C], e.g. the d_phase of one mkid_process_device call; j0 = the
 * number of phase rows processed before it since the last reset); d_events n wide packets
 * (28-bit stamps unwrapped into [j0 - 2^27, j0 + 2^27)); d_heights n floats. The context keeps
 * the last ncoeff rows it was given: when a call's j0 continues the previous call's rows, windows
 * that start before row j0 read them. NaN where the window is not inside (carried rows, rows).
 * In a streamed run that is the packets of a call's last (ncoeff - pre) rows: pass them again
 * with the next contiguous call (j0 = this call's j0 + rows) and their windows are then complete
 * (carried rows + new rows); the heights of a call are otherwise final.
 * Asynchronous on the context stream; device pointers only. */
int mkid_set_pulse_filter(mkid_ctx* ctx, const float* coeff, int32_t nch, int32_t ncoeff, int32_t pre);
int mkid_pulse_heights(mkid_ctx* ctx, const float* d_phase, int64_t rows, int64_t j0,
                       const uint64_t* d_events, int64_t n, float* d_heights);
/* The same with the packet count read on the device: min(*d_count, cap) packets, e.g. d_count =
 * &d_counts[1] of the mkid_process_device call that wrote d_events (no host round trip). */
int mkid_pulse_heights_counted(mkid_ctx* ctx, const float* d_phase, int64_t rows, int64_t j0,
                               const uint64_t* d_events, const int64_t* d_count, int64_t cap,
                               float* d_heights);

/* Kernel timing with HIP events on the context stream (for bench roofline numbers). */
#define MKID_K_CHANNELIZE 0
#define MKID_K_FIR_PHASE 1
#define MKID_K_TRIGGER 2
#define MKID_K_COMPACT 3
#define MKID_K_FRONT 4        /* fused K1-K6 (replaces CHANNELIZE + FIR_PHASE when used) */
#define MKID_K_COPY 5         /* mkid_stream_copy (measured HBM roof)                     */
#define MKID_K_HEIGHTS 6      /* mkid_pulse_heights                                       */
#define MKID_K_COUNT 7
/* mkid_set_timing: enable 0 off, any other value times every kernel (the round-1..3 meaning).
 * mkid_set_timing_mask: an OR of MKID_TIMING_ONLY(k) times only those kernels (0 = off). Each timed
 * launch records two events on the stream, and an event record costs a few microseconds of
 * stream time (rocprofv3 traces: 5-6 us gaps around timed kernels), so a throughput run times
 * only the kernel it reports. Both reset the accumulated times. */
#define MKID_TIMING_ONLY(k) (1 << (k))
int mkid_set_timing(mkid_ctx* ctx, int32_t enable);
int mkid_set_timing_mask(mkid_ctx* ctx, uint32_t kernel_mask);
int mkid_get_timing(mkid_ctx* ctx, int32_t kernel, double* total_ms, int64_t* launches);
const char* mkid_kernel_name(int32_t kernel);

/* Diagnostic, not on the hot path: HBM stream copy d_dst = d_src (bytes a multiple of 16, both
 * 16-byte aligned), device pointers, asynchronous on the context stream, timed as MKID_K_COPY.
 * bench.py reads the chip's achievable bandwidth from it in the same run. */
int mkid_stream_copy(mkid_ctx* ctx, void* d_dst, const void* d_src, int64_t bytes);

/* Synthetic ADC source for tests/bench (device; NOT part of the hot path):
 *   out[n] = base[(n0+n) mod 2^16] + AWGN(sigma) + sum_p amp_c e^{i theta_c(t)} (e^{i delta_p(t)} - 1)
 * base = conj(DAC tone comb) as int16 [2^16][2] (the loop-back spectrum inversion implied by
 * ROACH_Setup.py:485-487 vs 511-517); theta_c(t) = 2 pi (freq_index_c t mod 2^16)/2^16 + phase0_c;
 * delta_p(tau) = -amp_rad (1 - e^{-tau/tau_rise}) e^{-tau/tau_fall} for 0 <= tau < window (ADC
 * samples; shape after ReadoutControls/lib/pulses.py:470-472). pulses sorted by start. */
typedef struct mkid_synth_tone { float amp; float phase0; int32_t freq_index; int32_t pad; } mkid_synth_tone;
typedef struct mkid_pulse { int64_t start; int32_t tone; float amp_rad; } mkid_pulse;
int mkid_synth_adc(mkid_ctx* ctx, int16_t* d_out, int64_t nsamples, int64_t n0,
                   const int16_t* d_base_iq, const mkid_synth_tone* d_tones,
                   const mkid_pulse* d_pulses, int64_t npulses, float tau_rise, float tau_fall,
                   int32_t window, float noise_sigma, uint32_t seed);

#ifdef __cplusplus
}
#endif
#endif /* MKIDGPU_H */
