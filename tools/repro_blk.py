import sys, numpy as np
sys.path.insert(0, "/root/repo") if len(sys.argv) < 2 else sys.path.insert(0, sys.argv[1])
def rlp_len(n, off):
    if n < 56: return bytes([off+n])
    be=n.to_bytes((n.bit_length()+7)//8,'big'); return bytes([off+55+len(be)])+be
def rlp_bytes(b):
    if len(b)==1 and b[0]<0x80: return b
    return rlp_len(len(b),0x80)+b
def rlp_uint(x): return rlp_bytes(x.to_bytes(8,'big').lstrip(b'\0'))
def rlp_list(items):
    body=b''.join(items); return rlp_len(len(body),0xC0)+body
TO=b'\x22'*20
def geec_tx(nonce,data,is_geec,v,r,s):
    return rlp_list([rlp_uint(nonce),rlp_uint(1),rlp_uint(21000),rlp_bytes(TO),rlp_uint(7),rlp_bytes(data),bytes([1 if is_geec else 0x80]),rlp_uint(v),rlp_bytes(r),rlp_bytes(s)])
hdr=rlp_list([rlp_bytes(b'\0'*32),rlp_bytes(b'\x1d'*32),rlp_bytes(b'\x11'*20),rlp_uint(1),rlp_uint(8000000),rlp_list([]),rlp_uint(7)])
geec=[geec_tx(0,b'\x41'*23,True,0,b'',b'') for _ in range(3)]
import os
mode=os.environ.get("REPRO","geec_only")
if mode=="geec_only":
    blk=rlp_list([hdr,rlp_list([]),rlp_list(geec),rlp_list([]),rlp_list([]),rlp_list([])])
print(mode, len(blk), flush=True)
import eges_amd
eges_amd.init()
addr, st, counts, bst = eges_amd.block_senders_raw(blk, lists=0)
print("counts", counts, "bst", bst, flush=True)
