"""Extract the reference's recorded SoftGNSS tracking runs into a fixture.

Source: SCI/GLONASS/L1/trackingResults.dat and SCI/GLONASS/L2/trackingResults.dat
(POSTPROCESSING_SCILAB_RECEIVERS, written by postProcessing.sce:143 with
``save('trackingResults.dat', trackResults, settings, acqResults, channel)``).
They are decoded with oracle/scilab_save.py (no Scilab needed) and the values
the loop replay needs are stored as plain arrays in tests/golden/sgt_trackres.npz:

  <run>_<field>        trackResults(1).<field>, 1500 epochs (float64)
  <run>_settings       the numeric settings the loop uses (see SETTINGS)
  <run>_chan           [FCH, acquiredFreq, codePhase] of channel(1)

so the GPU box (no /root/reference) replays the same record.  Run from the repo
root: python tests/golden/make_sgt_trackres_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import scilab_save  # noqa: E402

SCI = "/root/reference/trunk/GNSS_SOFTWARE_RECEIVERS/POSTPROCESSING_SCILAB_RECEIVERS/GLONASS"
RUNS = ("L1", "L2")
FIELDS = ("absoluteSample", "codeFreq", "carrFreq", "I_E", "I_P", "I_L", "Q_E", "Q_P", "Q_L",
          "dllDiscr", "dllDiscrFilt", "pllDiscr", "pllDiscrFilt")
SETTINGS = ("samplingFreq", "codeFreqBasis", "codeLength", "IF", "L1_IF_step",
            "skipNumberOfBytes", "fileType", "dllCorrelatorSpacing", "dllNoiseBandwidth",
            "dllDampingRatio", "pllNoiseBandwidth", "fllNoiseBandwidth", "msToProcess")


def extract(path):
    d = scilab_save.load(path)
    tr = d["trackResults"][0]
    st = d["settings"]
    ch = d["channel"][0]
    out = {f: np.asarray(tr[f], dtype=np.float64).ravel() for f in FIELDS}
    out["settings"] = np.array([float(np.asarray(st[k]).ravel()[0]) for k in SETTINGS])
    out["chan"] = np.array([float(np.asarray(ch[k]).ravel()[0])
                            for k in ("FCH", "acquiredFreq", "codePhase")])
    return out


def main():
    arrays = {"settings_names": np.array(SETTINGS)}
    for run in RUNS:
        for k, v in extract(os.path.join(SCI, run, "trackingResults.dat")).items():
            arrays[f"{run}_{k}"] = v
    dst = os.path.join(ROOT, "tests", "golden", "sgt_trackres.npz")
    np.savez_compressed(dst, **arrays)
    print("wrote", dst)


if __name__ == "__main__":
    main()
