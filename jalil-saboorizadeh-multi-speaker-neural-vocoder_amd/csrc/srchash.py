"""Content hash of the HIP library's sources (csrc/*.hip, *.hpp, *.h, *.cpp and the C-ABI
header), 16 hex digits.  One definition for both sides: the Makefile compiles it into the
library (srnn_build_hash(), via build/build_hash.h) and samplernn_hip.lib() refuses a library
whose compiled-in hash differs from the tree's (a stale .so).

  python3 srchash.py            # prints the #define for build/build_hash.h
"""
import hashlib
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def csrc_hash(csrc=HERE):
    files = sorted(f for f in os.listdir(csrc) if f.endswith(('.hip', '.hpp', '.h', '.cpp')))
    h = hashlib.sha256()
    for f in files:
        h.update(f.encode())
        with open(os.path.join(csrc, f), 'rb') as fh:
            h.update(fh.read())
    hdr = os.path.join(os.path.dirname(os.path.dirname(csrc)), 'include', 'samplernn_hip.h')
    if os.path.exists(hdr):
        with open(hdr, 'rb') as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


if __name__ == '__main__':
    print('#define SRNN_BUILD_HASH "%s"' % csrc_hash())
