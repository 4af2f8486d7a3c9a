"""the unmodified reference chunkio, built by its own CMake
from a /tmp copy with cio-crc32 replaced by libchunkio_amd.so, passes its own
ctest 5/5 under every host CRC path (tools/ref_dropin_ctest.sh), with the
reference's own src/cio_sha1.c added to its source list and compiled unmodified
against include/sha1/sha1.h.

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
    # the reference's cio_sha1.c, built by its CMake against include/sha1/sha1.h,
    # takes SHA1_* from the shim and hashes like OpenSSL
    assert "U cioa_SHA1_Init" in out and "T cio_sha1_hash" in out
    assert "(hashlib a4a6313b9c8270616b062beacd02d8cca8e6619c)" in out
    assert "cio_sha1_hash(400kb.txt) = a4a6313b9c8270616b062beacd02d8cca8e6619c" in out
