"""How much brick walking the brick pass-through can remove (svo_cast.hip, skip_box PASS): C3 rays
(the C1 pose over the 4096^2 genWorld terrain, S = 16384) traced voxel by voxel in Python with
castRayFromCam's double DDA (src/ray_caster.cpp:54-87); each maximal run of voxels inside one mixed 4^3
brick is a brick visit.  A visit that does not end in a hit passes when no solid voxel of the brick lies
in the box spanned by its voxels.  usage: python tools/sim_brick_pass.py [rays]"""
import numpy as np, sys
sys.path.insert(0,'/root/repo')
import raytracing_test_amd as rt
H = np.asarray(rt.terrain_heights(4096, 4096)).reshape(4096,4096)
def solid(x,y,z):
    y &= 4095
    return 1 <= y <= H[x & 4095, z & 4095]
cache={}
def bm(b):
    if b not in cache:
        bx,by,bz=b; m=0
        for z in range(4):
            for y in range(4):
                for x in range(4):
                    if solid(bx*4+x,by*4+y,bz*4+z): m |= 1 << (z*16+y*4+x)
        cache[b]=m
    return cache[b]
def boxmask(lo,hi):
    m=0
    for z in range(lo[2],hi[2]+1):
        for y in range(lo[1],hi[1]+1):
            for x in range(lo[0],hi[0]+1):
                m |= 1 << (z*16+y*4+x)
    return m
W,Hh=1920,1080
cam=rt.normalize((1,-0.45,1))
dirs=rt.pixel_dirs(cam, W, Hh).reshape(-1,3)
rng=np.random.default_rng(1)
n=int(sys.argv[1]) if len(sys.argv)>1 else 1500
pix=rng.integers(0,W*Hh,n)
org=(4.0,90.0,4.0)
visits=skippable=steps_all=steps_skip=hitruns=0
for p in pix:
    d=dirs[p].astype(np.float32)
    step=[-1 if d[k]<0 else 1 for k in range(3)]
    delta=[float(np.float32(1.0)/d[k]) for k in range(3)]
    ad=[abs(x) for x in delta]
    r=[int(np.trunc(org[k])) for k in range(3)]
    ex=[org[k]-(1 if step[k]<0 else 0) for k in range(3)]
    T=[ad[k]-(ex[k]-r[k])*delta[k] for k in range(3)]
    S=16384; vox=[]; hit=False
    while S>0:
        S-=1
        if T[0]<T[1] and T[0]<T[2]: a=0
        elif T[1]<T[2]: a=1
        else: a=2
        r[a]+=step[a]; T[a]+=ad[a]
        vox.append(tuple(r))
        if solid(*r): hit=True; break
    # runs by brick
    i=0
    while i<len(vox):
        b=(vox[i][0]>>2,(vox[i][1]&4095)>>2,vox[i][2]>>2)
        j=i
        while j<len(vox) and (vox[j][0]>>2,(vox[j][1]&4095)>>2,vox[j][2]>>2)==b: j+=1
        m=bm(b)
        if m!=0 and m!=(1<<64)-1:
            visits+=1; L=j-i; steps_all+=L
            run=[(v[0]&3,v[1]&3,v[2]&3) for v in vox[i:j]]
            lo=[min(v[k] for v in run) for k in range(3)]; hi=[max(v[k] for v in run) for k in range(3)]
            if j==len(vox) and hit: hitruns+=1
            elif (boxmask(lo,hi) & m)==0:
                skippable+=1; steps_skip+=L
        i=j
print("rays %d brick visits/ray %.2f steps in bricks/ray %.2f hit-visits %.2f skippable visits %.3f (steps %.3f of brick steps)"%(n,visits/n,steps_all/n,hitruns/n,skippable/max(1,visits),steps_skip/max(1,steps_all)))
