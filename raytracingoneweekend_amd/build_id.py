"""Source hash baked into libottomarcher.so (om_build_id): sha256 over the library's sources
(csrc/*.hip, *.h, *.cpp, csrc/Makefile, include/*.h, sorted by path relative to the repo root,
each as `path\\0content\\0`), first 16 hex digits.  The csrc Makefile runs this file as a script
at link time; smoke() and tests/test_abi.py compare it with the id of the loaded library, so
a library built from other sources than the checked-out ones is caught.  No imports beyond
the standard library (it runs before the package can load)."""
import hashlib
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(_HERE)


def source_files(root=ROOT):
    csrc = os.path.join(root, "raytracingoneweekend_amd", "csrc")
    inc = os.path.join(root, "include")
    out = [os.path.join(csrc, f) for f in os.listdir(csrc)
           if f.endswith((".hip", ".h", ".cpp")) or f == "Makefile"]
    out += [os.path.join(inc, f) for f in os.listdir(inc) if f.endswith((".h", ".hpp"))]
    return sorted(out, key=lambda p: os.path.relpath(p, root))


def source_hash(root=ROOT):
    h = hashlib.sha256()
    for p in source_files(root):
        h.update(os.path.relpath(p, root).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read() + b"\0")
    return h.hexdigest()[:16]


if __name__ == "__main__":
    sys.stdout.write(source_hash())
