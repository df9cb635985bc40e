# LDS bank-conflict simulator for the attention tile accessors (MI355X guide LDS table)
B128 = [list(range(0,4))+list(range(12,16))+list(range(20,28)),
        list(range(4,12))+list(range(16,20))+list(range(28,32))]
B128 += [[l+32 for l in g] for g in B128]
def cycles(addrs, nbytes, groups, nbanks=64):
    tot=0
    for g in groups:
        banks={}
        for l in g:
            a=addrs[l]
            for w in range(nbytes//4):
                b=(a//4+w)%nbanks
                banks.setdefault(b,set()).add(a+4*w)
        tot+=max(len(v) for v in banks.values())
    return tot
def run(DP, off):
    # off(r, c16) -> byte offset of 16-B chunk c of row r
    worst={}
    # frag_rows
    for rbase in range(0,64,16):
        for ks in range(DP//32):
            addrs=[off(rbase+(l&15), ks*4+(l>>4)) for l in range(64)]
            worst['rows']=max(worst.get('rows',0),cycles(addrs,16,B128))
    # frag_tr (two reads a1 (rows rbase+4g+q) and a2 (+16 rows))
    for rbase in (0,32):
        for cbase in range(0,DP,16):
            for extra in (0,16):
                addrs=[]
                for l in range(64):
                    g,q,p=l>>4,(l>>2)&3,l&3
                    r=rbase+4*g+q+extra; col=cbase+4*p
                    addrs.append(off(r,col//8)+(col%8)*2)
                worst['tr']=max(worst.get('tr',0),cycles(addrs,8,[list(range(32)),list(range(32,64))]))
    # tile_store ds_write_b128: groups of 8 contiguous lanes, banks mod 32
    CPR=DP//8
    for j in range(64*DP//8//256):
        for w in range(4):
            addrs=[]
            for l in range(64):
                c=w*64+l+j*256; rr=c//CPR; ch=c%CPR
                addrs.append(off(rr,ch))
            worst['store']=max(worst.get('store',0),cycles(addrs,16,[list(range(i,i+8)) for i in range(0,64,8)],32))
    return worst
pad=lambda DP: (lambda r,c: r*(DP+8)*2+c*16)
F={0:0,1:2,2:3,3:1}
sw32=lambda r,c: r*64+((c^F[(r>>2)&3])*16)
sw64=lambda r,c: r*128+((c^(r&7))*16)
print('pad32',run(32,pad(32)),'(ideal rows 4, tr 2, store 8)')
print('pad64',run(64,pad(64)))
print('sw32',run(32,sw32))
print('sw64',run(64,sw64))
