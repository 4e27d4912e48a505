"""Generate tests/golden/e2e16368.json from the REFERENCE receiver at 16.368 Msps.

For each scenario of tests/e2e_scenarios.py (BASELINE configs 1 and 3), runs
oracle/_ref/e2e_ref_16368 -- the reference's own correlator.c, gp2021.c and
osgpsisr.c compiled from /root/reference with SAMP_RATE = 16.368e6 (make -C
oracle e2e16368) -- on the synthetic recording and stores the SHA-256 of the
IF file and of the per-call trace (REG_read words and loop state of every
channel, oracle/e2e_receiver.c), plus when each channel reached
CHANNEL_TRACKING.  The traces themselves are not stored (40-70 MB).

Usage:  python tests/golden/make_e2e16368_golden.py
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gnss-sdr.ru_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import gnsscorr as gc  # noqa: E402
import e2e_scenarios as E  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "e2e_ref_16368")


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "e2e16368"], check=True)
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for name, s in E.SCENARIOS.items():
            IF = E.make_if(gc, name)
            f_if, f_tr = os.path.join(d, "if.bin"), os.path.join(d, "tr.bin")
            IF.tofile(f_if)
            subprocess.run([REF, f_if, f_tr, str(s["calls"])] + [str(p) for p in s["prns"]],
                           check=True)
            tr = open(f_tr, "rb").read()
            out[name] = dict(calls=s["calls"], prns=s["prns"],
                             if_sha256=hashlib.sha256(IF.tobytes()).hexdigest(),
                             trace_sha256=hashlib.sha256(tr).hexdigest(),
                             tracking=E.summary(tr, len(s["prns"])))
            print(name, out[name]["tracking"])
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "e2e16368.json")
    json.dump(out, open(path, "w"), indent=1)


if __name__ == "__main__":
    main()
