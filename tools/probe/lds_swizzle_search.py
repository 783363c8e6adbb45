"""Bank-conflict model search for the attention backward's Q / dO piece images
(attention_x6.hip): cost of the staging stores (ds_write_b64: 4 groups of 16 contiguous lanes,
32 banks) and the 16-B fragment reads (ds_read_b128: the guide's 4 x 16-lane groups, 64 banks)
for chunk-XOR swizzles of the image rows; prints the best linear XOR swizzles.
``python tools/probe/lds_swizzle_search.py`` (CPU only)."""
import itertools
RSD = 36  # dwords per row
G128 = [list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
G128 = G128 + [[l+32 for l in g] for g in G128]
def read_cost(f):
    tot = 0
    for ks in range(4):
        for grp in G128:
            banks = {}
            for lane in grp:
                l32, h = lane & 31, lane >> 5
                c = (2*ks + h) ^ f(l32)
                a = l32*RSD + 4*c
                for d in range(4):
                    banks.setdefault((a+d) % 64, set()).add(a+d)
            tot += max(len(v) for v in banks.values())
    return tot  # cycles; ideal 4 per (ks) * 4 groups = 16
def write_cost(f):
    tot = 0
    for w in range(4):
        for rowsel in range(2):
            for g in range(4):
                banks = {}
                for lane in range(16*g, 16*g+16):
                    tid = 64*w + lane
                    sqp, sdq = tid & 15, tid >> 4
                    q = 2*sqp + rowsel
                    c = (sdq >> 1) ^ f(q)
                    a = q*RSD + 4*c + 2*(sdq & 1)
                    for d in range(2):
                        banks.setdefault((a+d) % 32, set()).add(a+d)
                tot += max(len(v) for v in banks.values())
    return tot  # ideal 1 per group: 4 w * 2 rows * 4 groups = 32

def main():
    cands = {'none': lambda q: 0, 'q>>4': lambda q: (q >> 4) & 1}
    for k in range(0, 5):
        for m in (1, 3, 7):
            for sh in (0, 1, 2):
                cands['((q>>%d)&%d)<<%d' % (k, m, sh)] = (lambda k, m, sh: (lambda q: (((q >> k) & m) << sh) & 7))(k, m, sh)
    cands['(q>>1)&7'] = lambda q: (q >> 1) & 7
    cands['((q>>1)&3)^((q>>3)&1)*4'] = lambda q: ((q >> 1) & 3) | (((q >> 3) & 1) << 2)
    cands['(q>>1)&7 rev'] = lambda q: ((q>>1)&1)<<2 | ((q>>2)&1)<<1 | ((q>>3)&1)
    res = sorted(((read_cost(f) / 16 + write_cost(f) / 32, read_cost(f), write_cost(f), n) for n, f in cands.items()))
    for r in res[:12]:
        print(r)
    print([r for r in res if r[3] in ('none', 'q>>4')])
    best = []
    for vs in itertools.product(range(8), repeat=5):
        def f(q, vs=vs):
            r = 0
            for i in range(5):
                if (q >> i) & 1: r ^= vs[i]
            return r
        rc = read_cost(f)
        if rc > 16: continue
        wc = write_cost(f)
        best.append((wc, rc, vs))
    best.sort()
    print(best[:5], len(best))


if __name__ == '__main__':
    main()
