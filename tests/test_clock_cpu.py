"""ClockStamps.digest: start / stop stamps are paired per CU (XCC id + HW_ID bits 8-15), so counters of
different CUs with unrelated offsets never mix (utils/profiler.py)."""
from deeplearning_mpi_amd.utils.profiler import ClockStamps


def _stamp(xcc, cu, mt, rt):
    return [xcc, cu << 8, mt, rt]


def test_clock_digest_pairs_per_cu():
    start, stop = [], []
    for xcc in range(8):
        for cu in range(4):
            off = (xcc * 7919 + cu * 104729) * 10 ** 6   # unsynchronised counter offsets
            mhz = 2000 + 50 * xcc
            rt0, rt1 = 10_000, 10_000 + 5_000_000          # 50 ms at 100 MHz
            start.append(_stamp(xcc, cu, off + rt0 * mhz // 100, rt0 + cu))
            stop.append(_stamp(xcc, cu, off + rt1 * mhz // 100, rt1 - cu))
    start.append(_stamp(0, 9, 5, 1))   # a CU stamped only at the start: ignored
    d = ClockStamps.digest([start, stop])
    assert d["xcds"] == 8 and d["cus"] == 32
    assert abs(d["sclk_mhz_min"] - 2000) < 1 and abs(d["sclk_mhz_max"] - 2350) < 1
    assert abs(d["sclk_mhz"] - 2175) < 1


def test_clock_digest_empty():
    assert ClockStamps.digest([[_stamp(0, 1, 5, 5)], [_stamp(1, 1, 9, 9)]]) is None
