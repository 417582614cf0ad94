#!/usr/bin/env python
"""Convert a Detectron weights pickle ({'blobs': {...}, 'cfg': ...},
detectron/utils/net.py:138-178) into the pickle-free .npz this build loads
by default.  Unpickling runs code from the file: only use on your own files.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == '__main__':
    from pps_amd import weights
    src, dst = sys.argv[1], sys.argv[2]
    blobs = weights.load_weights(src, trusted=True)
    weights.save_npz(dst, blobs)
    print('wrote %d blobs to %s' % (len(blobs), dst))
