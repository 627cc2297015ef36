"""Model of the octet kernels' B-fragment LDS reads (ds_read_b128 lane groups and
bank rule of MI355X_MICROARCH.md's LDS table) at the AlexNet b256 plans: the
fraction of LDS cycles that are bank conflicts, without and with the patch
segment shifts of x6.hip cbx6::seg_shift (round 5).  CPU only."""
G=[[0,1,2,3,12,13,14,15]+list(range(20,28)),[4,5,6,7,8,9,10,11,16,17,18,19,28,29,30,31]]
G+= [[l+32 for l in g] for g in G]
def cycles(addrs):
    tot=0
    for g in G:
        banks={}
        for l in g:
            a=addrs[l]
            for d in range(4):
                banks.setdefault((a//4+d)%64,set()).add(a//16)
        tot+=max(len(v) for v in banks.values())
    return tot
def geom(OW,Ho,pad,W,KH,shift):
    PW=W+2*pad; RPC=3*PW
    while (RPC-3*OW)%16: RPC+=1
    d=(3*OW*(1-KH))%16 if shift else 0
    return RPC,d
def sim(kind,OW,Ho,W,pad,KH,BN,NB,WC,N,tpi=0,shift=False):
    HW=OW*Ho; RPC,d=geom(OW,Ho,pad,W,KH,shift)
    tot=ideal=0
    ntiles=(N+BN-1)//BN if not tpi else (N//HW)*tpi
    for tn in range(min(ntiles,300)):
        if tpi: timg=tn//tpi; n0=timg*HW+(tn-timg*tpi)*BN; plast=min(n0+BN,(timg+1)*HW)-1
        else: n0=tn*BN; plast=min(n0+BN,N)-1
        img0=n0//HW; nseg=plast//HW-img0+1; f0=(n0-img0*HW)//OW
        sl=lambda s: (plast-(img0+s)*HW)//OW if s==nseg-1 else Ho-1
        p1=sl(0)-f0+KH; p2=p1+(sl(1)+KH if nseg>1 else 0); R=p2+(sl(2)+KH if nseg>2 else 0)
        octb=((R*RPC+2*d)*16+255)//256*256
        def addr(n,plane):
            n=n if n<=plast else (max(n0,n-((n-plast+15)&~15)) if shift else plast); img=n//HW; sp=n-img*HW; oh=sp//OW; ow=sp-oh*OW; sg=img-img0
            prow= oh-f0 if sg==0 else (p1 if sg==1 else p2)+oh
            return plane*octb+(prow*RPC+sg*d)*16+ow*48
        toff=lambda s:(s//KH)*RPC*16+(s%KH)*48
        for wc in range(WC):
            if kind=="cb":
                for j in range(NB):
                    base=[addr(n0+wc*32*NB+32*j+(l&31), l>>5) for l in range(64)]
                    for s in range(KH*KH):
                        tot+=cycles([a+toff(s) for a in base]); ideal+=4
            else:
                for j in range(2*NB):
                    base=[addr(n0+wc*32*NB+16*j+(l&15), (l>>4)&1) for l in range(64)]
                    for s0 in range(0,KH*KH-1,2):
                        tot+=cycles([base[l]+toff(s0+((l>>5)&1)) for l in range(64)]); ideal+=4
    return (tot-ideal)/tot
cfgs=[("conv2 cb16",("cb16",27,27,27,2,5,128,4,1,256*729,6)),
      ("conv3 cb",("cb",13,13,13,1,3,256,8,1,256*169)),
      ("conv4 cb",("cb",13,13,13,1,3,256,4,2,256*169)),
      ("conv5 cb16",("cb16",13,13,13,1,3,128,4,1,256*169))]
for name,a in cfgs:
    print(name,"conflict frac %.3f -> shifted + clamped %.3f"%(sim(*a),sim(*a,shift=True)))
