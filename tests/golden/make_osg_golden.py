"""Generate tests/golden/osg_<scenario>.npz from the REFERENCE correlator.

Runs every scenario of tests/osg_scenarios.py through the unmodified OSGPS
correlator.c + gp2021.c compiled from /root/reference (oracle/_ref/
libosg_ref.so, built by `make -C oracle ref`) and stores, per call, the full
REG_read register file plus the final gp2021_channel state.  The IF inputs are
NOT stored: the scenarios regenerate them with integer-only arithmetic.

Usage:  python tests/golden/make_osg_golden.py
"""
import ctypes as C
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import osg_oracle as oo  # noqa: E402
import osg_scenarios as S  # noqa: E402


def main():
    oo.build(ref=True)
    assert oo.have_ref(), "reference build missing"
    out_dir = os.path.dirname(os.path.abspath(__file__))
    for name in S.SCENARIOS:
        scn = S.get(name)
        ref = oo.RefOSG(12, scn["tic_period"])
        C.c_int.in_dll(ref.L, "use_iq_processing").value = 1 if scn["iq"] else 0
        ref.L.correlator_init(scn["tic_period"])
        regs, st = S.run(ref, scn)
        ifhash = hashlib.sha256(scn["IF"].tobytes()).hexdigest()
        np.savez_compressed(os.path.join(out_dir, f"osg_{name}.npz"), reg_read=regs,
                            carrier_phase=st["carrier_phase"], carrier_cycle=st["carrier_cycle"],
                            code_phase=st["code_phase"], half_chip=st["half_chip"],
                            acc=st["acc"], if_sha256=np.array(ifhash))
        print(name, regs.shape, "dump-calls", int((regs[:, 0x82] != 0).sum()), ifhash[:12])


if __name__ == "__main__":
    main()
