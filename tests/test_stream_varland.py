"""Host-side check that the framing DP's variable-message landing (stream.hip var_land: the
landing-or-terminal question restated with 32-bit positions, one bound for the buffer end and
the parse limit, and an early end for catch-up logs too long for what is left) equals the full
parse_var the walk and the emit use (binary.ReadVarint + the Unmarshal slice lengths,
minpaxosprotomarsh.go:126-153 / :352-387 / :470-507 / :648-672; paxosprotomarsh.go:152-176 /
:244-270 / :403-430), over ~14M variable-message positions of random and structured windows,
both wire formats, several buffer ends. Host code only (hipcc compiles the kernels alongside;
nothing runs on a GPU)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_var_land_equals_parse_var(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    exe = str(tmp_path / "var_land_check")
    subprocess.run([hipcc, "-O2", "-std=c++17", "--offload-arch=gfx950",
                    "-I", os.path.join(ROOT, "minpaxos_amd", "csrc"),
                    os.path.join(ROOT, "tools", "check", "var_land_check.cpp"), "-o", exe],
                   check=True, capture_output=True, timeout=600)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "var_land == parse_var" in r.stdout
