"""FAST compass-point early rejection: fraction of pixels / pixel pairs that pass the 4-point test
(necessary for a corner at threshold t) on the synthetic pyramids. CPU only."""
import sys, numpy as np
import os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, 'tests')); sys.path.insert(0, os.path.join(R, 'tools'))
import oracle_lib as O, synth
for preset in ("fr1","fr2","icl"):
    bgr, depth, _, cam = synth.sequence(2, seed=3, preset=preset)
    p = O.orb_params(1000)
    ref = O.pyramid(O.gray(bgr[0]), p)
    for l in (0,3,6):
        im = ref[l].astype(np.int16)
        h,w = im.shape
        v = im[3:h-3,3:w-3]
        c = [im[6:h,3:w-3], im[3:h-3,6:w], im[0:h-6,3:w-3], im[3:h-3,0:w-6]]
        d = [np.clip(v-x,0,None) for x in c]; b=[np.clip(x-v,0,None) for x in c]
        U = np.maximum.reduce([np.minimum(d[i],d[(i+1)%4]) for i in range(4)] + [np.minimum(b[i],b[(i+1)%4]) for i in range(4)])
        for t in (20,7):
            cand = U > t
            pair = cand[:, 0::2][:, :cand.shape[1]//2] | cand[:, 1::2][:, :cand.shape[1]//2]
            print(preset, l, t, "px cand %.3f pair cand %.3f" % (cand.mean(), pair.mean()))
