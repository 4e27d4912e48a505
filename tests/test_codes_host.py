"""CPU: code generators and host utilities (no GPU needed).

Known-answer tests: IS-GPS-200 Table 3-Ia "first 10 chips (octal)" for all 32
PRNs pins both the oracle restatement of generateCAcode.sci and the product's
gnsscorr_ca_code(); the OSGPS half-chip tables (correlator.c:63-91) carry the
same chip sequence; makeCaTable sampling rule; deterministic synthetic IF.
"""
import numpy as np
import pytest

import acq_oracle as A

ICD_OCTAL = [0o1440, 0o1620, 0o1710, 0o1744, 0o1133, 0o1455, 0o1131, 0o1454, 0o1626, 0o1504,
             0o1642, 0o1750, 0o1764, 0o1772, 0o1775, 0o1776, 0o1156, 0o1467, 0o1633, 0o1715,
             0o1746, 0o1763, 0o1063, 0o1706, 0o1743, 0o1761, 0o1770, 0o1774, 0o1127, 0o1453,
             0o1625, 0o1712]


def _octal(chips):
    bits = (np.asarray(chips[:10]) > 0).astype(int)
    return int("".join(map(str, bits)), 2)


@pytest.mark.parametrize("prn", range(1, 33))
def test_ca_first_chips_icd(gc, prn):
    assert _octal(A.generate_ca_code(prn)) == ICD_OCTAL[prn - 1]
    np.testing.assert_array_equal(gc.ca_code(prn), A.generate_ca_code(prn).astype(np.int8))


def test_ca_balance_and_autocorr(gc):
    for prn in (1, 17, 32):
        c = gc.ca_code(prn).astype(np.int64)
        assert c.sum() == -1 or c.sum() == 1  # Gold codes: 512 ones / 511 zeros
        ac = np.array([np.dot(c, np.roll(c, k)) for k in range(1, 1023)])
        assert set(np.unique(ac)) <= {-65, -1, 63}


def test_st_code(gc):
    st = gc.st_code()
    np.testing.assert_array_equal(st, A.generate_st_code().astype(np.int8))
    ac = np.array([np.dot(st.astype(int), np.roll(st.astype(int), k)) for k in range(1, 511)])
    assert (ac == -1).all()  # m-sequence


def test_osg_tables_carry_icd_codes(oracle):
    o = oracle.OracleOSG()
    img = o.table_image()
    off_e = 2 * (2046 * 33 + 2)
    for prn in range(1, 33):
        early_even = img[off_e + prn * 2046: off_e + prn * 2046 + 2046: 2]
        np.testing.assert_array_equal(early_even, A.generate_ca_code(prn).astype(np.int8))


@pytest.mark.parametrize("fs", [16.368e6, 16.0e6, 4.092e6])
def test_sample_code_matches_make_ca_table(gc, fs):
    n = int(round(fs / 1000.0))
    for prn in (1, 9):
        np.testing.assert_array_equal(gc.sample_code(gc.ca_code(prn), 1.023e6, fs, n),
                                      A.make_ca_table_row(prn, fs, n))
    np.testing.assert_array_equal(gc.sample_code(gc.st_code(), 0.511e6, fs, n),
                                  A.make_st_table_row(fs, n))


def test_ifgen_deterministic_and_levels(gc):
    sig = [dict(system=0, prn=3, code_phase=10.0, doppler=1500.0, cn0=45.0)]
    a = gc.ifgen(20000, sig, seed=1)
    b = gc.ifgen(20000, sig, seed=1)
    c = gc.ifgen(20000, sig, seed=2)
    np.testing.assert_array_equal(a, b)
    assert not np.array_equal(a, c)
    assert set(np.unique(a)) <= {-3, -1, 1, 3}


def test_acq_oracle_finds_planted_signal(gc):
    fs = 16.368e6
    IF = gc.ifgen(2 * 16368, [dict(system=0, prn=5, code_phase=300.0, doppler=2250.0, cn0=48.0)],
                  fs=fs, seed=9)
    freqs = A.gps_bins(2.42e6, 10)          # 21 bins @ 500 Hz
    codes = np.stack([A.make_ca_table_row(p, fs) for p in (5, 6)])
    res = A.acquire(IF, fs, codes, freqs, np.tile(np.arange(len(freqs)), (2, 1)))
    # 300 chips of code phase at t=0 -> the replica must be delayed by 1023-300 chips
    assert abs(res[0]["code_phase"] - 1 - (1023 - 300) * 16) <= 1
    assert abs(res[0]["carr_freq"] - (2.42e6 + 2250)) <= 250
    assert res[0]["metric"] > 2.5 and res[1]["metric"] < res[0]["metric"]


def test_sdr_prn_spectra_range(gc):
    """sdr_strong_kernel multiplies by the negated Q of the PRN spectra in int16
    (sdr_acq.hip cmulsc_d2): the table (prn_codes.h values, gen_fft_codes.m
    scaling to 2^9) must stay within +-502, far from -32768."""
    pc = gc.sdr_prn_codes().astype(np.int32)
    assert np.abs(pc).max() <= 502
