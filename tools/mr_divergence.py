"""MirrorRefraction 1080p: how much of the secondary-ray chain a wave runs for lanes that
have finished. Traces each pixel's reflect/refract chain with the oracle's closest-hit
(oracle/oracle.py closest, numpy reflect/refract in fp64: an estimate of chain depths,
not a parity path), then compares per 8x8 tile (one wave) the levels the wave executes
(max lane depth) with the useful lane-levels / 64, and with a 256-pixel block that
compacts its live rays per level. Reference: provided/scene.py:97-111, 189-209."""
import sys; sys.path[:0]=['/root/repo','/root/repo/python-raytracer_amd']
import numpy as np, json
import rtx
from oracle import oracle as O
W,H=1920,1080
sc = rtx.load_bundled_scene("MirrorRefraction", resolution=(W,H))
vc = sc.vc
d, base = O.load_bundle("MirrorRefraction", resolution=[W,H])
os_ = O.OracleScene(d, base)
mt = {m['ID']: m.get('type','diffuse') for m in d['materials']}
eta = {m['ID']: m.get('refr_index',1.0) for m in d['materials']}
xs = vc.left + (0.5+np.arange(W))*(vc.right-vc.left)/W
ys = vc.bottom + (0.5+np.arange(H))*(vc.top-vc.bottom)/H
u,v,w = [np.asarray(a,np.float64) for a in (vc.u,vc.v,vc.w)]
X,Y = np.meshgrid(xs, ys[::-1])   # row 0 = top
dirs = X[...,None]*u + Y[...,None]*v - w
dirs /= np.linalg.norm(dirs,axis=-1,keepdims=True)
o = np.broadcast_to(np.asarray(vc.position,np.float64), dirs.shape).reshape(-1,3).copy()
dd = dirs.reshape(-1,3).copy()
n = W*H
depth = np.zeros(n, np.int32)
shade = np.zeros((10, n), bool)  # pixel shades a hit at this level
alive = np.ones(n, bool); inside = np.zeros(n,bool)
for level in range(10):
    idx = np.nonzero(alive)[0]
    if len(idx)==0: break
    depth[idx] += 1
    t, ob, sb, m, nn, pp = os_.closest(0.0, o[idx], dd[idx])
    hit = ob >= 0
    shade[level, idx[hit]] = True
    types = np.array([mt.get(int(k),'diffuse') if k>=0 else 'none' for k in m])
    cont = hit & ((types=='mirror')|(types=='refractive'))
    newo = o[idx].copy(); newd = dd[idx].copy()
    for k in np.nonzero(cont)[0]:
        D = dd[idx[k]]; N = nn[k].astype(np.float64); P = pp[k].astype(np.float64)
        if types[k]=='mirror':
            r = D - 2*np.dot(N,D)*N; newo[k] = P + 0.01*r; newd[k]=r; inside[idx[k]]=False
        else:
            e = eta[int(m[k])]; ins = inside[idx[k]]
            if ins: N=-N; e_ = e
            else: e_ = 1.0/e
            c = np.dot(N,D); kk = 1 - e_*e_*(1-c*c)
            if kk < 0: cont[k]=False; continue
            r = e_*D - (e_*c + np.sqrt(kk))*N
            newo[k]=P+1e-4*r; newd[k]=r; inside[idx[k]] = not ins
    o[idx]=newo; dd[idx]=newd
    alive[idx] = cont
dep = depth.reshape(H,W)
tiles = dep.reshape(H//8,8,W//8,8).transpose(0,2,1,3).reshape(-1,64)
wave_levels = tiles.max(1).sum()
lane_levels = tiles.sum()/64
print("pixels depth hist", np.bincount(depth))
print("wave-levels %d  useful(lane-levels/64) %.0f  ratio %.3f" % (wave_levels, lane_levels, wave_levels/lane_levels))
# block of 4 waves (256 px) compaction: per block, levels beyond 0 compacted
blk = tiles.reshape(-1,4,64)
comp = 0
for b in blk:
    comp += 4  # level 0
    for L in range(2, 11):
        k = (b >= L).sum()
        comp += int(np.ceil(k/64))
sh = shade.reshape(10, H//8, 8, W//8, 8).transpose(0, 1, 3, 2, 4).reshape(10, -1, 64)
print("shading: wave-levels %d  useful %.0f  ratio %.3f" % (sh.any(2).sum(), sh.sum() / 64, sh.any(2).sum() / (sh.sum() / 64)))
print("with block compaction: wave-levels %d ratio %.3f" % (comp, comp/lane_levels))
