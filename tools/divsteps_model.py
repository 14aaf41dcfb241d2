#!/usr/bin/env python3
"""CPU models of the latency kernels' scalar-ALU divsteps (modinv_row.cuh), used to design and
check divsteps_30_var_asm:

  - divsteps_c: the compiled C loop (divsteps_30_var_c: 12-bit Newton inverse at every swap);
  - divsteps_asm: an instruction-by-instruction model of the assembly loop (two role-exchanged
    copies, 6-bit cancellation cap, sentinel mask) with 32-bit wrap semantics;
  - stats: iterations, divsteps, swaps and the limit histogram of full inversions mod n and p.

`python tools/divsteps_model.py` checks the two loops equal on random (eta, f, g) and prints the
statistics."""
import collections
import random
import sys
M32=0xffffffff
def s32(x):
    x&=M32; return x-(1<<32) if x>>31 else x
def ff1(x):
    x&=M32
    return (x & -x).bit_length()-1 if x else -1
def divsteps_c(eta,f0,g0):
    u,v,q,r=1,0,0,1; f,g=f0,g0; i=30
    x=f; x=(x*(2-f*x))&M32; x=(x*(2-f*x))&M32; nx=(-x)&M32
    while True:
        zeros=ff1(g | ((M32<<i)&M32))
        g=(g>>zeros)&M32; u=(u<<zeros)&M32; v=(v<<zeros)&M32; eta-=zeros; i-=zeros
        if i==0: break
        if eta<0:
            eta=-eta; tf,tu,tv=f,u,v; f=g; u=q; v=r; g=(-tf)&M32; q=(-tu)&M32; r=(-tv)&M32
            x=f; x=(x*(2-f*x))&M32; x=(x*(2-f*x))&M32; nx=(-x)&M32
        limit=min(eta+1,i); limit=min(limit,12)
        m=M32>>(32-limit)
        w=(g*nx)&m
        g=(g+f*w)&M32; q=(q+u*w)&M32; r=(r+v*w)&M32
    return eta,(s32(u),s32(v),s32(q),s32(r))
def divsteps_asm(eta,f0,g0):
    A,B,uA,vA,uB,vB,sm=f0,g0,1,0,0,1,0xC0000000
    copy='A'
    while True:
        if copy=='A':
            z=ff1(B|sm); B=(B>>z)&M32; uA=(uA<<z)&M32; vA=(vA<<z)&M32; eta-=z; sm=(s32(sm)>>z)&M32
            if sm==M32: return eta,(s32(uA),s32(vA),s32(uB),s32(vB))
            if eta<0:
                eta=-eta; A=(-A)&M32; uA=(-uA)&M32; vA=(-vA)&M32
                copy='B'  # falls into LB_tail
                # LB_tail
                t=min(eta+1,6); m=((1<<t)-1)&~sm&M32
                tmp=(B*B-2)*B*A &M32; w=tmp&m
                A=(A+B*w)&M32; uA=(uA+uB*w)&M32; vA=(vA+vB*w)&M32
                continue
            # LA_tail
            t=min(eta+1,6); m=((1<<t)-1)&~sm&M32
            tmp=(A*A-2)*A*B&M32; w=tmp&m
            B=(B+A*w)&M32; uB=(uB+uA*w)&M32; vB=(vB+vA*w)&M32
        else:
            z=ff1(A|sm); A=(A>>z)&M32; uB=(uB<<z)&M32; vB=(vB<<z)&M32; eta-=z; sm=(s32(sm)>>z)&M32
            if sm==M32: return eta,(s32(uB),s32(vB),s32(uA),s32(vA))
            if eta<0:
                eta=-eta; B=(-B)&M32; uB=(-uB)&M32; vB=(-vB)&M32
                copy='A'
                t=min(eta+1,6); m=((1<<t)-1)&~sm&M32
                tmp=(A*A-2)*A*B&M32; w=tmp&m
                B=(B+A*w)&M32; uB=(uB+uA*w)&M32; vB=(vB+vA*w)&M32
                continue
            t=min(eta+1,6); m=((1<<t)-1)&~sm&M32
            tmp=(B*B-2)*B*A&M32; w=tmp&m
            A=(A+B*w)&M32; uA=(uA+uB*w)&M32; vA=(vA+vB*w)&M32
def check(count=200000):
  rnd=random.Random(5)
  bad=0
  for k in range(count):
    f=rnd.getrandbits(32)|1; g=rnd.getrandbits(32); eta=rnd.randint(-40,40)
    if divsteps_c(eta,f,g)!=divsteps_asm(eta,f,g):
        bad+=1
  return bad

N=0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
P=2**256-2**32-977
def sim(M,x):
    # libsecp modinv var (eta convention), batches of 30, count inner iterations and divsteps
    f,g=M,x; eta=-1; iters=0; steps=0; batches=0
    while g!=0:
        batches+=1
        i=30; fl=f&0xffffffff; gl=g&0xffffffff
        u,v,q,r=1,0,0,1
        while True:
            zeros=min(((gl|(1<<i)) & -(gl|(1<<i))).bit_length()-1, i)
            gl>>=zeros; u<<=zeros; v<<=zeros; eta-=zeros; i-=zeros; steps+=zeros
            if i==0: break
            iters+=1
            if eta<0:
                eta=-eta; fl,gl=gl,(-fl); u,v,q,r=q,r,-u,-v
            limit=min(eta+1,i,12)
            m=(1<<limit)-1
            w=(gl*(-pow(fl,-1,1<<32)))&m
            gl+=fl*w; q+=u*w; r+=v*w
        # apply
        f,g=(u*f+v*g)>>30,(q*f+r*g)>>30
    return iters,steps,batches
def stats():
 for M,name in ((N,'n'),(P,'p')):
    tot=[0,0,0]; K=300
    for _ in range(K):
        a,b,c=sim(M,random.randrange(1,M))
        tot[0]+=a; tot[1]+=b; tot[2]+=c
    print(name,'iters',tot[0]/K,'divsteps',tot[1]/K,'batches',tot[2]/K)

def sim2(M,x):
    f,g=M,x; eta=-1; iters=0; swaps=0; lims=[]
    while g!=0:
        i=30; fl=f&0xffffffff; gl=g&0xffffffff
        u,v,q,r=1,0,0,1
        while True:
            zeros=min(((gl|(1<<i)) & -(gl|(1<<i))).bit_length()-1, i)
            gl>>=zeros; u<<=zeros; v<<=zeros; eta-=zeros; i-=zeros
            if i==0: break
            iters+=1
            if eta<0:
                swaps+=1
                eta=-eta; fl,gl=gl,(-fl); u,v,q,r=q,r,-u,-v
            limit=min(eta+1,i,12); lims.append(limit)
            m=(1<<limit)-1
            w=(gl*(-pow(fl,-1,1<<32)))&m
            gl+=fl*w; q+=u*w; r+=v*w
        f,g=(u*f+v*g)>>30,(q*f+r*g)>>30
    return iters,swaps,lims
def swap_stats():
    K=200; it=0; sw=0; L=collections.Counter()
    for _ in range(K):
        a,b,l=sim2(N,random.randrange(1,N)); it+=a; sw+=b; L.update(l)
    print('iters',it/K,'swaps',sw/K, 'limit hist', sorted((k,round(v/K,1)) for k,v in L.items()))


if __name__ == "__main__":
    bad = check()
    print("asm model vs C loop, 200000 random (eta, f, g):", bad, "mismatches")
    stats()
    swap_stats()
    sys.exit(1 if bad else 0)
