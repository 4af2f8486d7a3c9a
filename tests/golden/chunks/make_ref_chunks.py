#!/usr/bin/env python3
"""Recipe for tests/golden/chunks/: chunk files written, damaged and loaded by
the REFERENCE chunkio (fixture data only; see gen_ref_chunks.c).

  1. the reference built by its own CMake from a /tmp copy
     (tools/ref_dropin_ctest.sh; reused when already there),
  2. gcc gen_ref_chunks.c against that build's libchunkio-static.a and
     libcio-crc32.a (the reference's own deps/crc32),
  3. run it into a scratch directory; keep the final files under files/ and
     a manifest.json holding, per file, the operations performed, the damage
     applied, the reference loader's verdict, the file's size and SHA-256, and
     the SHA-256 of the file as the reference's load left it (a legacy length
     is written back on load).

Runs in the build container only (needs /root/reference, cmake, gcc).
Usage: python tests/golden/chunks/make_ref_chunks.py
"""
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))
REF = "/root/reference"
WORK = "/tmp/cioa_ref_dropin"


def sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def main():
    stock = os.path.join(WORK, "stock")
    if not os.path.exists(os.path.join(stock, "build", "src", "libchunkio-static.a")):
        subprocess.run([os.path.join(ROOT, "tools", "ref_dropin_ctest.sh"), WORK], check=True,
                       stdout=subprocess.DEVNULL)
    b = os.path.join(stock, "build")
    exe = os.path.join(tempfile.mkdtemp(prefix="gen_ref_chunks_"), "gen_ref_chunks")
    subprocess.run(["gcc", "-O1", "-Wall", "-o", exe, os.path.join(HERE, "gen_ref_chunks.c"),
                    f"-I{stock}/include", f"-I{b}/include", f"-I{stock}/deps", f"-I{stock}/deps/monkey/include",
                    f"{b}/src/libchunkio-static.a", f"{b}/deps/crc32/libcio-crc32.a"], check=True)
    out = tempfile.mkdtemp(prefix="ref_chunks_")
    r = subprocess.run([exe, out], check=True, capture_output=True, text=True)
    scen = json.loads(r.stdout)
    files = os.path.join(HERE, "files")
    shutil.rmtree(files, ignore_errors=True)
    os.makedirs(files)
    for s in scen:
        src = os.path.join(out, "root", "s", s["name"])
        shutil.copyfile(src, os.path.join(files, s["name"]))
        s["size"] = os.path.getsize(src)
        s["sha256"] = sha(src)
        s["sha256_after_load"] = sha(os.path.join(out, "load", "s", s["name"]))
    man = {
        "generator": "tests/golden/chunks/gen_ref_chunks.c via make_ref_chunks.py",
        "reference_build": "fluent/chunkio 1.5.4, its own CMake (CIO_DEV=On) in a /tmp copy; "
                           "libchunkio-static.a + deps/crc32 libcio-crc32.a",
        "pattern": "content byte i of (len, seed) = ((i * 131 + seed * 7 + 17) % 251) + 1",
        "stream": "s",
        "chunks": scen,
    }
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(man, f, indent=1)
        f.write("\n")
    shutil.rmtree(out)
    shutil.rmtree(os.path.dirname(exe))
    for s in scen:
        ld = s["load"]
        print(f"{s['name']:26s} {s['size']:7d} B  load ok={ld['ok']!s:5s} err={ld['err']:3d} "
              f"last_chunk_error={ld['last_chunk_error']:4d} "
              + (f"crc_cur={ld['crc_cur']:#010x} content={ld['content_size']}" if ld["ok"] else "")
              + ("  (changed by load)" if s["sha256_after_load"] != s["sha256"] else ""))


if __name__ == "__main__":
    sys.exit(main())
