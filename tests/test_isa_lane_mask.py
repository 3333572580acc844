"""The code-generation pattern behind the round-5 K3 stalls of two diagnostic
builds -- register copies of wave-wide values placed
where the wave runs with a partial or empty lane mask -- is absent from every
in-tree code object, and the checker (tools/isa_lane0_check.py) finds both
of its forms in small hand-written listings shaped like the two stalled
objects."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_lane0_check as chk  # noqa: E402

# the stage-split object: copies inside a barrier arrival's lane-0 branch
P2_CASE = """_Zk:
\tv_lshl_add_u32 v113, v73, 2, s0
\ts_mov_b64 s[0:1], exec
\ts_and_b64 s[2:3], s[0:1], s[2:3]
\ts_mov_b64 exec, s[2:3]
\tds_add_rtn_u32 v28, v76, v84 offset:35312
\tv_mov_b32_e32 v56, v73
\ts_or_b64 exec, exec, s[0:1]
\tv_lshlrev_b64 v[72:73], v70, s[18:19]
\tv_mov_b32_e32 v73, v56
\tds_read_b32 v0, v113 offset:16
.Lfunc_end0:
"""
# the trace+check object: copies after a poll loop's exit, before the restore
P1_CASE = """_Zk:
\ts_and_saveexec_b64 s[6:7], s[36:37]
\ts_mov_b64 s[20:21], 0
\tds_read_b32 v37, v82 offset:35932
\ts_waitcnt lgkmcnt(0)
\tv_cmp_le_u32_e64 s[36:37], s23, v37
\ts_or_b64 s[20:21], s[36:37], s[20:21]
\ts_andn2_b64 exec, exec, s[20:21]
\ts_cbranch_execnz 65527
\tv_mov_b32_e32 v61, v91
\ts_or_b64 exec, exec, s[6:7]
\tv_mov_b32_e32 v91, v61
.Lfunc_end0:
"""
# the epoch-priority object: a live-range split inside an else arm, undone
# after the join's exec restore
P3_CASE = """_Zk:
\tv_cmp_eq_u32_e32 vcc, 3, v9
\ts_and_saveexec_b64 s[2:3], vcc
\ts_xor_b64 s[0:1], exec, s[2:3]
\tv_mov_b32_e32 v74, 1
\ts_andn2_saveexec_b64 s[0:1], s[0:1]
\tv_mov_b32_e32 v74, 2
\tv_mov_b32_e32 v87, v73
\ts_or_b64 exec, exec, s[0:1]
\tv_mov_b32_e32 v73, 0
\tv_mov_b32_e32 v73, v87
.Lfunc_end0:
"""
# a phi written in both arms is not a split
PHI = """_Zk:
\ts_and_saveexec_b64 s[8:9], s[62:63]
\ts_xor_b64 s[42:43], exec, s[8:9]
\tv_cndmask_b32_e64 v48, v14, v46, s[62:63]
\ts_andn2_saveexec_b64 s[42:43], s[42:43]
\tv_mov_b32_e32 v48, v14
\ts_or_b64 exec, exec, s[42:43]
\tv_mov_b32_e32 v14, v48
.Lfunc_end0:
"""
CLEAN = """_Zk:
\ts_mov_b64 s[0:1], exec
\ts_and_b64 s[2:3], s[0:1], s[2:3]
\ts_mov_b64 exec, s[2:3]
\tv_mov_b32_e32 v1, 1
\tds_write_b32 v76, v1 offset:34084
\ts_or_b64 exec, exec, s[0:1]
.Lfunc_end0:
"""


def test_checker_finds_both_patterns():
    assert chk.check_text(P2_CASE, "p2") == 1
    assert chk.check_text(P1_CASE, "p1") == 1
    assert chk.check_text(P3_CASE, "p3") == 1
    assert chk.check_text(PHI, "phi") == 0
    assert chk.check_text(CLEAN, "clean") == 0


LIBS = sorted(glob.glob(os.path.join(ROOT, "libwebp_amd", "libwebp_amd*.so")))


@pytest.mark.skipif(not LIBS or not os.path.exists(chk.LLVM + "llvm-objdump"),
                    reason="no built library / ROCm llvm tools")
@pytest.mark.parametrize("lib", LIBS, ids=[os.path.basename(p) for p in LIBS])
def test_code_objects_clean(lib):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_lane0_check.py"), lib],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:]
