"""The built library's LDS-DMA destinations (M0) come from SGPRs defined on every path to the DMA
(tools/check_lds_dma.py; VERDICT r05 item 6, DESIGN §4 "LDS-DMA destinations and hipcc's switch
lowering").  CPU-only: disassembles the gfx950 code objects of libkdlae.so, no GPU call."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "rethink_acoustic_image_enhancement_amd", "libkdlae.so")


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="needs the built library and llvm-objdump")
def test_every_lds_dma_m0_is_defined_on_every_path():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_lds_dma.py"), LIB],
                       capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "kernels with LDS DMA checked" in r.stdout
