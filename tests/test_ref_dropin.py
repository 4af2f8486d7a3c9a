"""the unmodified reference chunkio, built by its own CMake
from a /tmp copy with cio-crc32 replaced by libchunkio_amd.so, passes its own
ctest 5/5 under every host CRC path (tools/ref_dropin_ctest.sh).

Boundary evidence only (the oracle is oracle/_ref).  Needs the reference
tree and cmake, so it runs in the build container and skips on the GPU box,
where /root/reference does not exist."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "CMakeLists.txt")) or shutil.which("cmake") is None,
                    reason="needs /root/reference and cmake (build container only)")
def test_reference_ctest_passes_against_the_shim(tmp_path):
    work = tmp_path / "ref_dropin"
    r = subprocess.run([os.path.join(ROOT, "tools", "ref_dropin_ctest.sh"), str(work)],
                       capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert out.rstrip().endswith("DROPIN_CTEST_OK"), out[-4000:]
    # 5/5 as shipped, then 5/5 on each of the three host CRC paths
    assert out.count("100% tests passed") == 4, out[-4000:]
    for t in ("cio-test-fs", "cio-test-metadata_update", "cio"):
        assert f"{t}" in out and "NOT LINKED" not in out
    assert "U crc_update" in out
