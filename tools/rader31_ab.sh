# bash tools/rader31_ab.sh -> the radix-31 A/B (direct symmetric vs Rader) on the GPU,
# plus the fp64 VALU instruction counts of one 31-point transform from the ISA
set -e
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/rader31_ab.hip -o /tmp/rader31_ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S tools/rader31_ab.hip -o /tmp/rader31_ab.s
python3 - <<'PY'
import re
txt = open("/tmp/rader31_ab.s").read()
for form in ("0", "1"):
    m = re.search(r"^(_Z3k31ILi%s\w*):(.*?)\.Lfunc_end" % form, txt, re.S | re.M)
    body = m.group(2)
    import collections
    ops = collections.Counter(re.sub(r"_e(32|64)$", "", o) for o in re.findall(r"^\s*(v_\w+)", body, re.M))
    cnt = {k: ops.get(k, 0) for k in ("v_fmac_f64", "v_fma_f64", "v_add_f64", "v_mul_f64",
                                       "v_readlane_b32", "v_writelane_b32")}
    cnt["fp64"] = sum(v for k, v in ops.items() if k.endswith("_f64"))
    cnt["all_valu"] = sum(ops.values())
    vg = re.search(r"NumVgprs:\s*(\d+)", txt[m.end():]).group(1)
    print("direct" if form == "0" else "rader ", "per kernel (one transform in the loop body):", cnt, "VGPRs", vg)
PY
timeout -k 10 120 /tmp/rader31_ab 64
