#!/usr/bin/env python3
"""Register / spill / scratch metadata of every kernel in the gfx950 code object of a built object file (the
llvm-readelf notes tests/test_build_flags.py reads), one line per kernel; optional name filter.

    python3 tools/co_meta.py mahi-mpc_amd/build/lane_kernels.o [ExoArm]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_build_flags import _kernel_metadata  # noqa: E402

obj = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for name, v in sorted(_kernel_metadata(obj).items()):
    if flt in name:
        print(f"{name[:110]:110s} vspill {v.get('vgpr_spill_count')} sspill {v.get('sgpr_spill_count')} "
              f"scratch {v.get('private_segment_fixed_size')}")
