"""Host-side AddressSanitizer + UBSan run of the PowerSGD plan builder (csrc/plan.cpp)
over random model shapes / ranks, with the kernels' table invariants checked
(tools/asan/plan_fuzz.cpp; GPU ASan is not available, so sanitizers cover host code)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or not os.path.isdir("/opt/rocm/include"), reason="needs g++ + ROCm headers")
def test_plan_builder_under_asan_ubsan(tmp_path):
    exe = tmp_path / "plan_fuzz"
    csrc = os.path.join(ROOT, "network_distributed_pytorch_amd", "csrc")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-I" + csrc,
           os.path.join(ROOT, "tools", "asan", "plan_fuzz.cpp"), os.path.join(csrc, "plan.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    # verify_asan_link_order=0: the environment may preload other libraries ahead of ASan
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    out = subprocess.run([str(exe), "150"], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "plan_fuzz ok" in out.stdout
