"""Photon-packet wire path downstream of the device trigger.

The firmware's packet stage (K8) writes time-ordered 64-bit packets into a pair of 2^14-word
BRAMs (`pulses_bram0` = low words, `pulses_bram1` = high words) with a write pointer
`pulses_addr`, and marks every second of the 1 PPS timebase with an all-ones end-of-second word
(channel field 255). On each ROACH, PulseServer ships the ring to PacketMaster in 8192-word halves
(PulseServer.c:151-227 `wait_for_write_position`, 318-386 `send_packet`); PacketMaster bins the
packets per pixel per second into `/r<roach>/p<pixel>/t<start>` variable-length rows
(PacketMaster.c:245-405 main loop, 921-1050 layout and `write_sec_data`).

This module restates that path on the host, fed by the device's wide packets:

* `Timebase`      phase row -> (second, microsecond since PPS) for an integer sample clock;
* `WireStream`    wide device packets of successive process calls -> the time-ordered wire stream
                  (reference 64-bit packets, timestamps in us since PPS, end-of-second markers);
* `PulseRing`     the pulses_bram0/1 + pulses_addr ring the shim's readPulses reads;
* `PulseServer`   the half-ring shipping rule of PulseServer.c;
* `PacketMaster`  per-pixel/per-second binning with the reference's 2500-event cap semantics.

Build decisions (the firmware is absent, .MISSING_LARGE_BLOBS:1-27): the stream's first ADC
sample after a reset is a PPS edge; phase row j is at ADC sample j*N; packets are ordered by
stamped row, then channel; the end-of-second marker of second k follows the last packet stamped
in second k; startBuffer 0 -> 1 restarts the ring at address 0.
"""
import numpy as np

from . import codecs

END_OF_SECOND = 0xFFFFFFFFFFFFFFFF     # PacketMaster.c:331-337: adr 255, packet == (uint64_t)-1
RING_WORDS = 1 << 14                   # pulses_bram0/1 depth (ROACH_Pulses.py:799-800)
HALF_WORDS = 8192                      # PulseServer.c:159 FIRST_HALF; PacketMaster.c:44 BUFSIZE_INTS
FIRST_HALF_ENDPTR = 8500               # PulseServer.c:160
SECOND_HALF_ENDPTR = 300               # PulseServer.c:161
MAX_EVENTS_PER_SEC = 2500              # PacketMaster.c:55
TS_BITS = 20                           # reference packet time field: us since PPS (< 2^20)


class Timebase:
    """1 PPS timebase of one feedline: phase row j (ADC sample j*N at fs, fs an integer number of
    samples per second) lies in second (j N) // fs at microsecond ((j N) mod fs) 10^6 // fs."""

    def __init__(self, fs, N):
        if float(fs) != int(fs) or int(fs) <= 0:
            raise ValueError('the sample clock must be a positive integer number of S/s')
        self.fs = int(fs)
        self.N = int(N)

    def second(self, rows):
        return (np.asarray(rows, np.int64) * self.N) // self.fs

    def microsecond(self, rows):
        s = np.asarray(rows, np.int64) * self.N
        return ((s % self.fs) * 1000000) // self.fs

    def first_row(self, sec):
        """First phase row of second `sec` (ceil(sec fs / N))."""
        return (int(sec) * self.fs + self.N - 1) // self.N


def unwrap_stamps(ts, j0):
    """28-bit device stamps of one call whose phase rows start at global row j0 -> global rows.
    A call's packets are stamped in [j0 - 1, j0 + rows - 1) (the peak is the sample before the
    one that emits the packet)."""
    ts = np.asarray(ts, np.int64)
    base = int(j0) - 1
    return base + ((ts - base) % (1 << 28))


def encode_wire(ch, peak, base, us, wide=False):
    """Packet fields -> 64-bit wire words. Reference layout (C <= 254):
    ch 8b | peak 12b | p1 = peak-base+2048 12b | base 12b | us 20b (ROACH_Pulses.py:805-832);
    wide layout (any C): the device's wide packet with the time field in us since PPS."""
    ch = np.asarray(ch, np.uint64)
    peak = np.asarray(peak, np.int64)
    base = np.asarray(base, np.int64)
    us = np.asarray(us, np.uint64)
    if wide:
        return ((ch << np.uint64(52)) | (peak.astype(np.uint64) << np.uint64(40)) |
                (base.astype(np.uint64) << np.uint64(28)) | us)
    if np.any(ch >= 255):
        raise ValueError('reference packets have an 8-bit channel field (255 = end of second)')
    p1 = np.clip(peak - base + 2048, 0, 4095).astype(np.uint64)
    return ((ch << np.uint64(56)) | (peak.astype(np.uint64) << np.uint64(44)) | (p1 << np.uint64(32)) |
            (base.astype(np.uint64) << np.uint64(20)) | (us & np.uint64((1 << TS_BITS) - 1)))


class WireStream:
    """Wide device packets of successive process calls -> the firmware's time-ordered wire stream.

    push(wide, j0, rows) takes the packets of one call that covered global phase rows
    [j0, j0 + rows) and returns the words now final: every packet of each second that is complete
    (no later call can still stamp a packet in it), ordered by stamped row then channel, each
    second closed by one END_OF_SECOND word. Seconds without packets still get their marker."""

    def __init__(self, fs, N, wide=False):
        self.tb = Timebase(fs, N)
        self.wide = wide
        self.next_sec = 0                       # first second not yet closed
        self.dropped = 0                        # packets of channels >= 255 (reference layout)
        self._rows = np.zeros(0, np.int64)      # held packets (global rows) ...
        self._words = np.zeros(0, np.uint64)    # ... and their wide words

    def push(self, wide_packets, j0, rows):
        w = np.asarray(wide_packets, np.uint64)
        r = unwrap_stamps(w & np.uint64(codecs.PKT_TS_MASK), j0)
        self._rows = np.concatenate([self._rows, r])
        self._words = np.concatenate([self._words, w])
        # packets stamped <= j_end - 2 are final (a packet at row r is emitted at row r + 1)
        final_row = int(j0) + int(rows) - 2
        out = []
        while self.tb.first_row(self.next_sec + 1) <= final_row + 1:
            lim = self.tb.first_row(self.next_sec + 1)
            sel = self._rows < lim
            out.append(self._encode(self._rows[sel], self._words[sel]))
            out.append(np.array([END_OF_SECOND], np.uint64))
            self._rows, self._words = self._rows[~sel], self._words[~sel]
            self.next_sec += 1
        return np.concatenate(out) if out else np.zeros(0, np.uint64)

    def _encode(self, rows, words):
        f = codecs.unpack_wide(words)
        if not self.wide:
            # the reference's 8-bit channel field cannot carry channels >= 255 (255 marks the
            # end of a second): such packets are counted and left out of the wire stream
            keep = f['ch'] < 255
            self.dropped += int((~keep).sum())
            rows = rows[keep]
            f = {k: v[keep] for k, v in f.items()}
        o = np.lexsort((f['ch'], rows))
        return encode_wire(f['ch'][o], f['peak'][o], f['base'][o], self.tb.microsecond(rows[o]), self.wide)


class PulseRing:
    """pulses_bram0 (low words) / pulses_bram1 (high words) ring of 2^14 entries and the write
    pointer pulses_addr (index of the next entry written), as read by readPulses
    (ROACH_Pulses.py:796-832) and PulseServer (PulseServer.c:43-45)."""

    def __init__(self):
        self.bram0 = np.zeros(RING_WORDS, np.uint32)
        self.bram1 = np.zeros(RING_WORDS, np.uint32)
        self.addr = 0
        self.written = 0            # total words written since the last restart

    def start_buffer(self, on, prev=0):
        if on and not prev:         # startBuffer 0 -> 1 (PulseServer.c:78-80) restarts the ring
            self.addr = 0
            self.written = 0

    def write(self, words):
        w = np.asarray(words, np.uint64)
        lo = (w & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        hi = (w >> np.uint64(32)).astype(np.uint32)
        idx = (self.addr + np.arange(len(w))) % RING_WORDS
        self.bram0[idx] = lo       # later writes to the same slot win (numpy: last index wins)
        self.bram1[idx] = hi
        self.addr = (self.addr + len(w)) % RING_WORDS
        self.written += len(w)

    def read(self, name, size, offset=0):
        """Big-endian BRAM bytes, as the katcp read / the /proc ioreg files return them."""
        b = self.bram0 if name == 'pulses_bram0' else self.bram1
        return b.astype('>u4').tobytes()[offset:offset + size]


class PulseServer:
    """PulseServer.c's shipping rule over a PulseRing: wait_for_write_position (151-227) reads
    the pointer once on entry; started in the first half it ships the first half once the pointer
    passes 8500, started in the second half it ships the second half once the pointer has wrapped
    past 300; send_packet (318-386) then sends 32 KiB of low words followed by 32 KiB of high
    words from that half. poll() plays one pointer check."""

    def __init__(self, ring):
        self.ring = ring
        self._arm()

    def _arm(self):
        start = self.ring.addr
        self.first = start < HALF_WORDS
        self.end = FIRST_HALF_ENDPTR if self.first else SECOND_HALF_ENDPTR
        self.require_wrap = not self.first

    def poll(self):
        p = self.ring.addr
        if p > self.end and (not self.require_wrap or p < HALF_WORDS):
            off = 0 if self.first else HALF_WORDS * 4
            low = self.ring.read('pulses_bram0', HALF_WORDS * 4, off)
            high = self.ring.read('pulses_bram1', HALF_WORDS * 4, off)
            self._arm()
            return low, high
        return None


def serve(words, ring=None, server=None, poll_every=256):
    """Write wire words into the ring as the firmware would, letting PulseServer poll the pointer
    after every `poll_every` words; returns the (low, high) 32 KiB block pairs it shipped."""
    ring = ring if ring is not None else PulseRing()
    server = server if server is not None else PulseServer(ring)
    sent = []
    w = np.asarray(words, np.uint64)
    for i in range(0, len(w), poll_every):
        ring.write(w[i:i + poll_every])
        blk = server.poll()
        if blk is not None:
            sent.append(blk)
    return sent


class PacketMaster:
    """PacketMaster.c's per-pixel/per-second binning (main loop 245-405, write_sec_data 978-1050):
    blocks of 8192 (low, high) network-order words per roach; adr = high >> 24; adr 255 closes the
    roach's current second (a marker other than all-ones is counted as corrupted but still closes
    it); a photon of pixel adr < n_pixels is appended to that pixel's list for the second, of
    which only the first MAX_EVENTS_PER_SEC - 1 are kept (the reference keeps writing the overflow
    into one spare slot that is never stored); other adr values are counted as non-pixel photons.
    Seconds at or beyond exptime are ignored. `rows[(r, p)][sec]` is the VL row the reference
    writes to /r<r>/p<p>/<dataset>; `photon_counts[sec][r * n_pixels + p]` its quick-look count."""

    def __init__(self, n_roaches, n_pixels, exptime, dataset='t0', max_events=MAX_EVENTS_PER_SEC):
        self.R, self.P, self.exptime = int(n_roaches), int(n_pixels), int(exptime)
        self.dataset = dataset
        self.keep = int(max_events) - 1
        self.sec = [0] * self.R
        self._open = [[[] for _ in range(self.P)] for _ in range(self.R)]
        empty = np.zeros(0, np.uint64)
        self.rows = {(r, p): [empty] * self.exptime for r in range(self.R) for p in range(self.P)}
        self.photon_counts = np.zeros((self.exptime, self.R * self.P), np.int64)
        self.corrupted_eos = 0
        self.nonpixel = 0

    def names(self):
        return ['/r%d/p%d/%s' % (r, p, self.dataset) for r in range(self.R) for p in range(self.P)]

    def done(self):
        return all(s >= self.exptime for s in self.sec)

    def receive(self, r, low_block, high_block):
        lo = np.frombuffer(low_block, '>u4').astype(np.uint64)
        hi = np.frombuffer(high_block, '>u4').astype(np.uint64)
        pk = (hi << np.uint64(32)) | lo
        adr = (hi >> np.uint64(24)).astype(np.int64)
        eos = np.flatnonzero(adr == 255)
        start = 0
        for e in list(eos) + [len(pk)]:
            if self.sec[r] >= self.exptime:
                return
            seg_adr, seg_pk = adr[start:e], pk[start:e]
            ok = seg_adr < self.P
            self.nonpixel += int((~ok).sum())
            for p in np.unique(seg_adr[ok]):
                self._open[r][p].append(seg_pk[ok & (seg_adr == p)])
            if e < len(pk):
                if pk[e] != np.uint64(END_OF_SECOND):
                    self.corrupted_eos += 1
                self._close_second(r)
            start = e + 1

    def _close_second(self, r):
        s = self.sec[r]
        for p in range(self.P):
            parts = self._open[r][p]
            row = np.concatenate(parts)[:self.keep] if parts else np.zeros(0, np.uint64)
            self.rows[(r, p)][s] = row
            self.photon_counts[s, r * self.P + p] = len(row)
            self._open[r][p] = []
        self.sec[r] = s + 1


def decode_wire(words, wide=False):
    """Wire words -> dict of fields (reference layout unless wide); END_OF_SECOND entries get
    ch = 255 (reference) / 4095 (wide)."""
    w = np.asarray(words, np.uint64)
    if wide:
        return dict(ch=((w >> np.uint64(52)) & np.uint64(0xFFF)).astype(np.int64),
                    peak=((w >> np.uint64(40)) & np.uint64(0xFFF)).astype(np.int64),
                    base=((w >> np.uint64(28)) & np.uint64(0xFFF)).astype(np.int64),
                    us=(w & np.uint64((1 << 28) - 1)).astype(np.int64))
    return dict(ch=(w >> np.uint64(56)).astype(np.int64),
                peak=((w >> np.uint64(44)) & np.uint64(0xFFF)).astype(np.int64),
                p1=((w >> np.uint64(32)) & np.uint64(0xFFF)).astype(np.int64),
                base=((w >> np.uint64(20)) & np.uint64(0xFFF)).astype(np.int64),
                us=(w & np.uint64(0xFFFFF)).astype(np.int64))
