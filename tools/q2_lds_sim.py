"""CPU model of q2_lds_kernel's data flow (csrc/backtr.hip): one wave per
sweep group, chunks in a per-workgroup LDS ring, handed down through global
memory by each workgroup's lowest wave, with the kernel's waits.  Random
interleavings of the waves (generators that yield at every wait and between
loads and stores) must give exactly the level-by-level order's result for a
stand-in block operator (a fixed random 63 x 63 matrix per block).  Found the
round-6 first draft's bug: the top wave did not carry the incoming chunk's
last row (i = 63, outside the block's 63 rows) into the ring.
    python tools/q2_lds_sim.py"""
# CPU simulation of q2_lds_kernel v2's data flow (random interleavings).
import numpy as np, random, sys
QB=32; QW=8; RS=16
def ntasks(n,j): return (n-3-j)//32+1 if j<=n-3 else 0
def run(n, k, seed, buggy=False):
    rng=np.random.default_rng(seed)
    ng2=-(-(n-2)//32); Z0=rng.standard_normal((n,k))
    # block op: rows rb0..rb0+62 (<n): F <- M_{G2,s} F with a random 63x63 matrix whose row/col 63 unused
    mats={}
    def op(G2,s,F):
        key=(G2,s)
        if key not in mats: mats[key]=np.eye(63)+0.1*np.random.default_rng(hash(key)%2**32).standard_normal((63,63))
        return mats[key]@F
    # reference: level order
    Zr=Z0.copy(); smax=ntasks(n,0)
    nlev=smax+ng2-1
    for L in range(nlev):
        for s_ in range(smax):
            G2=ng2-1-(L-s_)
            if G2<0 or G2>=ng2 or s_>=ntasks(n,32*G2): continue
            rb0=32*G2+1+32*s_; r1=min(n,rb0+63)
            F=np.zeros((63,k)); F[:r1-rb0]=Zr[rb0:r1]
            F=op(G2,s_,F); Zr[rb0:r1]=F[:r1-rb0]
    # kernel sim
    Zg=Z0.copy(); Wq=-(-ng2//QW)
    lds=[np.zeros((RS,32,k)) for _ in range(Wq)]
    done=[[0]*QW for _ in range(Wq)]; gprog=[0]*(ng2+1)
    for w in range(Wq):
        for q in range(QW):
            c=w*QW+q
            for r in range(32):
                row=32*c+1+r
                if row<n: lds[w][c%RS][r]=Z0[row]
    def wave(w,g):
        G0=w*QW; G2=G0+g; gtop=min(QW,ng2-G0)-1
        if g>gtop: return
        nb=ntasks(n,32*G2); nbu=ntasks(n,32*(G2+1)) if G2+1<ng2 else 0
        for s_ in range(nb):
            c=G2+s_; rb0=32*c+1
            if nbu>0:
                need=min(s_+1,nbu)
                if g<gtop:
                    while done[w][g+1]<need: yield
                else:
                    while gprog[G2+1]<need: yield
            from_g = g==gtop
            if from_g:
                prev=c+1-RS-G0
                if prev>=0:
                    while done[w][0]<prev+1: yield
            F=np.zeros((63,k)); x63=None
            for i in range(64):
                row=rb0+i; r=i&31; ch=c if i<32 else c+1
                if i>=32 and from_g: v=Zg[min(row,n-1)].copy()
                else: v=lds[w][ch%RS][r].copy()
                if i<63 and row<n: F[i]=v
                if i==63: x63=v
            yield
            F=op(G2,s_,F)
            last = s_+1==nb
            if (not buggy) and from_g and not (g==0 and last) and rb0+63<n:
                lds[w][(c+1)%RS][31]=x63
            for i in range(63):
                row=rb0+i
                if row>=n: continue
                r=i&31; ch=c if i<32 else c+1
                gl = g==0 and (i<32 or last)
                if gl: Zg[row]=F[i]
                else: lds[w][ch%RS][r]=F[i]
            done[w][g]=s_+1
            if g==0: gprog[G2]=s_+1
            yield
    gens=[wave(w,g) for w in range(Wq) for g in range(QW)]
    gens=[x for x in gens if x is not None]
    rnd=random.Random(seed)
    alive=list(gens)
    steps=0
    while alive:
        gi=rnd.randrange(len(alive))
        try: next(alive[gi])
        except StopIteration: alive.pop(gi)
        steps+=1
        if steps>10**7: raise RuntimeError("deadlock?")
    return np.abs(Zg-Zr).max()


def main():
    for n in [64, 100, 600, 1000, 1025, 2049]:
        for seed in range(3):
            print(n, seed, run(n, 3, seed))
    print("without the last-row carry:", run(600, 3, 0, buggy=True))


if __name__ == "__main__":
    main()
