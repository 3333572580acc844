"""Debug helper: parse the VP8 frame header of a .webp (RFC 6386 section
9.2-9.11) up to the token probability updates and the skip flag, to compare
two encoders' partition-0 decisions. Not used by the product or the tests."""
import os
import re

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# coefficient update probabilities, parsed from vp8_tables.h
src=open(os.path.join(_ROOT, 'libwebp_amd/csrc/vp8_tables.h')).read()
i=src.index('kVP8CoeffUpdateProba'); j=src.index('};',i)
upd=[int(x) for x in re.findall(r'\d+', src[src.index('=',i):j])]
assert len(upd)==1056, len(upd)
class BD:
    def __init__(s,b): s.b=b; s.pos=0; s.value=0; s.range=255; s.bits=-8; s.fill()
    def fill(s):
        while s.bits < 0:
            s.value = (s.value << 8) | (s.b[s.pos] if s.pos < len(s.b) else 0); s.pos+=1; s.bits += 8
    def get(s, p):
        split = 1 + (((s.range - 1) * p) >> 8)
        bigsplit = split << s.bits
        if s.value >= bigsplit:
            s.range -= split; s.value -= bigsplit; bit=1
        else:
            s.range = split; bit=0
        while s.range < 128:
            s.range <<= 1; s.bits -= 1
            s.fill() if s.bits < 0 else None
        return bit
    def lit(s,n):
        v=0
        for _ in range(n): v=(v<<1)|s.get(128)
        return v
def parse(data):
    i=data.index(b'VP8 ')+8
    d=data[i:]
    tag=d[0]|(d[1]<<8)|(d[2]<<16); p0=tag>>5
    bd=BD(d[10:10+p0])
    out={}
    bd.lit(1); bd.lit(1)
    seg=bd.lit(1); out['seg']=seg
    if seg:
        upm=bd.lit(1); upd_data=bd.lit(1)
        if upd_data:
            bd.lit(1)
            for _ in range(4):
                if bd.lit(1): bd.lit(7); bd.lit(1)
            for _ in range(4):
                if bd.lit(1): bd.lit(6); bd.lit(1)
        if upm:
            for _ in range(3):
                if bd.lit(1): bd.lit(8)
    out['ftype']=bd.lit(1); out['flevel']=bd.lit(6); out['sharp']=bd.lit(3)
    if bd.lit(1):
        if bd.lit(1):
            for _ in range(8):
                if bd.lit(1): bd.lit(6); bd.lit(1)
    out['parts']=bd.lit(2)
    out['q']=bd.lit(7)
    for _ in range(5):
        if bd.lit(1): bd.lit(4); bd.lit(1)
    bd.lit(1)
    n=0
    for k in range(1056):
        if bd.get(upd[k]): bd.lit(8); n+=1
    out['updates']=n
    out['skip']=bd.lit(1)
    if out['skip']: out['skip_p']=bd.lit(8)
    return out
