"""TEST INFRASTRUCTURE ONLY (never imported by mkids_sdr_amd/ or bench's timed region).

Per-packet pure-Python restatement of the photon-packet wire path, written
loop-for-loop after the reference C programs so that mkids_sdr_amd.packets (vectorised numpy) can
be checked against it:

* firmware K8 wire stream: time-ordered packets with us-since-PPS stamps and an all-ones
  end-of-second word per second (build decisions listed in mkids_sdr_amd/packets.py; the reference
  packet layout is ROACH_Pulses.py:805-832 / PacketMaster.c:291-292);
* PulseServer.c:151-227 wait_for_write_position + 318-386 send_packet (half-ring shipping);
* PacketMaster.c:304-397 (per-word loop) + 978-1023 (write_sec_data rows).

Parity: the reference C programs need sockets, /proc ioreg files and HDF5 (absent), so they are
not run; this restatement follows their text (parity pinned to the source, not to outputs).
"""

EOS = (1 << 64) - 1
RING = 1 << 14
FIRST_HALF = 8192
FIRST_HALF_ENDPTR = 8500
SECOND_HALF_ENDPTR = 300


def wire_stream(packets, fs, N, rows_done):
    """packets: list of (row, ch, peak, base) with global stamped rows; the stream has processed
    phase rows < rows_done. Returns the wire words of every complete second, each closed by EOS."""
    fs = int(fs)
    out = []
    pk = sorted(packets, key=lambda t: (t[0], t[1]))
    sec = 0
    while True:
        lim = ((sec + 1) * fs + N - 1) // N           # first row of second sec + 1
        if lim > rows_done - 1:                        # row lim - 1 may still get a packet
            break
        for row, ch, peak, base in pk:
            if (row * N) // fs == sec:
                us = ((row * N) % fs) * 1000000 // fs
                p1 = min(max(peak - base + 2048, 0), 4095)
                out.append((ch << 56) | (peak << 44) | (p1 << 32) | (base << 20) | (us & 0xFFFFF))
        out.append(EOS)
        sec += 1
    return out


def pulse_server(words, poll_every=256):
    """Firmware writes `words` into the 2^14 ring from address 0 (startBuffer 0 -> 1); the server
    checks the pointer after every poll_every words. Returns the shipped (low, high) word lists."""
    bram0 = [0] * RING
    bram1 = [0] * RING
    addr = 0
    sent = []

    def arm(start):
        if start < FIRST_HALF:                          # PulseServer.c:174-178
            return FIRST_HALF_ENDPTR, 0, 1
        return SECOND_HALF_ENDPTR, 1, 0                 # :180-184

    end_ptr, require_wrap, first_half = arm(addr)
    for i in range(0, len(words), poll_every):
        for w in words[i:i + poll_every]:
            bram0[addr] = w & 0xFFFFFFFF
            bram1[addr] = w >> 32
            addr = (addr + 1) % RING
        ptr = addr
        if ptr > end_ptr and (require_wrap == 0 or ptr < FIRST_HALF):   # :214-218
            seek = 0 if first_half == 1 else FIRST_HALF                   # :338-339
            sent.append((bram0[seek:seek + FIRST_HALF], bram1[seek:seek + FIRST_HALF]))
            end_ptr, require_wrap, first_half = arm(addr)
    return sent


def packet_master(blocks, n_pixels, exptime, max_events=2500):
    """blocks: list of (low words, high words) of ONE roach in arrival order. Returns
    (rows[pixel][sec] lists, photon_counts[sec][pixel], corrupted, nonpixel)."""
    plist = [0] * n_pixels
    photons = [[0] * max_events for _ in range(n_pixels)]
    rows = [[[] for _ in range(exptime)] for _ in range(n_pixels)]
    counts = [[0] * n_pixels for _ in range(exptime)]
    sec = 0
    corrupted = nonpixel = 0
    for low, high in blocks:
        for j in range(len(low)):                      # PacketMaster.c:304
            packet = (high[j] << 32) | low[j]
            adr = high[j] >> 24
            if sec < exptime:                          # :329
                if adr == 255:                         # :331
                    if packet != EOS:
                        corrupted += 1
                    for i in range(n_pixels):          # write_sec_data :1012-1023
                        rows[i][sec] = photons[i][:plist[i]]
                        plist[i] = 0                   # :357-360
                    sec += 1                           # :362
                else:
                    if adr < n_pixels:                 # :371
                        idx = plist[adr]
                        photons[adr][idx] = packet     # :373-374
                        if plist[adr] < max_events - 1:   # :375
                            plist[adr] += 1
                            counts[sec][adr] += 1
                    else:
                        nonpixel += 1                  # :382-386
    return rows, counts, corrupted, nonpixel
