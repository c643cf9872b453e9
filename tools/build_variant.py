"""Build a tuning variant of libctr_hip.so with extra -D flags on chosen sources.

    python tools/build_variant.py NAME SOURCE[,SOURCE] -DFLAG=VAL ...

Writes rl_ctr_prediction_amd/variants/lib_NAME.so (travels to the GPU box like the main
library); select it with CTR_HIP_LIB=<path>. Tuning only — the product loads libctr_hip.so.
"""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from rl_ctr_prediction_amd import build_lib as B  # noqa: E402

name, srcs, flags = sys.argv[1], sys.argv[2].split(","), sys.argv[3:]
B.build()
out = ROOT / "rl_ctr_prediction_amd" / "variants"
out.mkdir(exist_ok=True)
vb = B.BUILD.parent / f"variant_{name}"
vb.mkdir(parents=True, exist_ok=True)
objs = []
for s in B.SOURCES:
    obj = B.BUILD / (s.rsplit(".", 1)[0] + ".o")
    if s in srcs:
        obj = vb / obj.name
        subprocess.run([B._hipcc(), *B.CXXFLAGS, *flags, "-c", str(B.CSRC / s), "-o", str(obj)],
                       check=True)
    objs.append(str(obj))
subprocess.run([B._hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o",
                str(out / f"lib_{name}.so"), *objs], check=True)
print(out / f"lib_{name}.so")
