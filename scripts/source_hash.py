#!/usr/bin/env python3
"""Hash of the sources the renderer library is built from (sphereflake-raytracer_amd/csrc/*, its Makefile
and include/sphereflake/sf.h), in a fixed order. The Makefile embeds it in the library (sf_build_id); bench.py
compares the embedded hash with the tree's, so a bench line or a profile names exactly the sources of the
library that produced it.

  source_hash.py                 print the 16-hex-digit hash
  source_hash.py --header PATH   write `#define SF_SOURCE_HASH "<hash>"` to PATH if it changed
"""
import hashlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "sphereflake-raytracer_amd")


def source_files():
    csrc = os.path.join(PKG, "csrc")
    files = sorted(os.path.join(csrc, f) for f in os.listdir(csrc) if not f.startswith("."))
    return files + [os.path.join(PKG, "Makefile"), os.path.join(REPO, "include", "sphereflake", "sf.h")]


def source_hash():
    h = hashlib.sha256()
    for p in source_files():
        h.update(os.path.relpath(p, REPO).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


if __name__ == "__main__":
    v = source_hash()
    if len(sys.argv) > 2 and sys.argv[1] == "--header":
        text = f'#define SF_SOURCE_HASH "{v}"\n'
        try:
            with open(sys.argv[2]) as f:
                if f.read() == text:
                    sys.exit(0)
        except OSError:
            pass
        with open(sys.argv[2], "w") as f:
            f.write(text)
    else:
        print(v)
