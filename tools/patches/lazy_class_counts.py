import sys
p=sys.argv[1]; s=open(p).read()
old='''    const unsigned nbk = (unsigned)(v.nb[0] * v.nb[1] * v.nb[2]);
    unsigned ncls[kMaxBatch];
    int total = 0;
#pragma unroll
    for (int c = 0; c < kMaxBatch; ++c) {
        ncls[c] = min(coh_load(&count[c + 1]), nbk);
        total += (int)ncls[c];
    }
    int c = kMaxBatch - 1;
    unsigned k0 = 0;  // list ordinal where class c starts (classes visited in descending order)'''
new='''    const unsigned nbk = (unsigned)(v.nb[0] * v.nb[1] * v.nb[2]);
    int total = 0;
#pragma unroll
    for (int c = 0; c < kMaxBatch; ++c) total += (int)min(coh_load(&count[c + 1]), nbk);
    int c = kMaxBatch - 1;
    unsigned k0 = 0;  // list ordinal where class c starts (classes visited in descending order)
    // the length of class c only (one scalar live across the items; the next class's is read when
    // the walk reaches it -- at most kMaxBatch - 1 times per wave)
    unsigned nc = min(coh_load(&count[c + 1]), nbk);'''
assert old in s; s=s.replace(old,new)
old='''            while (c > 0 && (unsigned)k - k0 >= ncls[c]) k0 += ncls[c--];'''
new='''            while (c > 0 && (unsigned)k - k0 >= nc) {
                k0 += nc;
                --c;
                nc = min(coh_load(&count[c + 1]), nbk);
            }'''
assert old in s; s=s.replace(old,new)
old='''        while (c > 0 && k - k0 >= ncls[c]) k0 += ncls[c--];'''
new='''        while (c > 0 && k - k0 >= nc) {
            k0 += nc;
            --c;
            nc = min(coh_load(&count[c + 1]), nbk);
        }'''
assert old in s; s=s.replace(old,new)
open(p,'w').write(s)
