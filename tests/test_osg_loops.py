"""CPU: the OSG loop constants and start state of the GPU channel loops.

Reference: osgnss_next_step.c:99-107 (init_tracking_loops_parameter) (calc_* / convert_* in osgpsisr.c:253-330),
correlator.c:110-121 (reference words), osgnss_next_step.c:73-84 (reset).
"""
import ctypes as C
import os

import numpy as np
import pytest

import gnsscorr as gc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libosg_ref.so")


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref not built")
def test_constants_equal_reference():
    L = C.CDLL(REF_SO)
    out = (C.c_long * 8)()
    L.ref_isr_constants(out)
    c = gc.osg_loop_cfg()
    assert [c.fll_i1, c.fll_i2, c.fll_i3, c.dll_i1, c.dll_i2, c.carrier_ref, c.code_ref,
            c.d_freq] == list(out)


def test_reset_state_and_register_words():
    c = gc.osg_loop_cfg()
    loops, cmds = gc.osg_loop_reset(c, [27, 0, 5])
    assert (loops["state"] == 1).all() and (loops["del_freq"] == 1).all()
    assert (loops["search_max_prn_delay"] == 2045).all() and (loops["search_max_f"] == 5).all()
    assert list(cmds["prn"]) == [27, 0, 5]
    # gp2021.c ch_carrier / ch_code: (f << (32 - bits)) * 5 in 32 bits
    assert (cmds["carrier_incr"] == ((c.carrier_ref << 2) * 5) & 0xFFFFFFFF).all()
    assert (cmds["code_incr"] == ((c.code_ref << 3) * 5) & 0xFFFFFFFF).all()
    assert (cmds["epoch_load"] == 0).all() and (cmds["slew"] == 0).all()
