"""bench.py's detector block (`detector_score`): packets of the last step matched against the
injected pulses, the unmatched ones histogrammed by their delay after the channel's previous pulse
and by the channel's attenuation / loop fraction. Hand-built packets, CPU only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _pkt(ch, row):
    return (np.uint64(ch) << np.uint64(52)) | np.uint64(row)


def test_detector_score_bins_unmatched_packets():
    N = 8
    # channel 0: pulses at rows 100 and 5000; channel 1: a pulse at row 300
    ps = np.array([100 * N, 300 * N + 3, 5000 * N])
    pt = np.array([0, 1, 0])
    ev = np.array([_pkt(0, 101),      # matches the row-100 pulse
                   _pkt(0, 250),      # 150 rows after it: a tail re-fire
                   _pkt(0, 2000),     # 1900 rows after it: a noise trigger
                   _pkt(1, 10),       # before channel 1's only pulse
                   _pkt(1, 301),      # matches
                   _pkt(0, 5001)], np.uint64)
    d = bench.detector_score(ev, 0, ps, pt, N, atten=np.array([2.0, 17.0]), loop_R=np.array([0.1, 0.9]))
    assert d['packets'] == 6 and d['pulses'] == 3
    assert d['unmatched_packets'] == 3
    assert d['unmatched_per_pulse'] == 1.0
    h = d['unmatched_delay_rows']
    assert h['no_earlier_pulse'] == 1 and h['100-199'] == 1 and h['1000-inf'] == 1
    assert sum(h.values()) == 3
    assert {e['atten_db'][0]: e['packets'] for e in d['unmatched_by_atten_db']} == {0: 2, 15: 1}
    assert [e['packets'] for e in d['unmatched_by_loop_R']] == [2, 0, 0, 1]
    assert d['isolated'] == 3 and d['exactly_one_frac'] == 1.0
