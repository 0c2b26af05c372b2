import csv,collections,re,sys
for d in sys.argv[1:]:
    r=list(csv.DictReader(open(d+'/run_kernel_trace.csv')))
    def short(n):
        m=re.search(r'(bn_\w+(<\w+>)?|dconv_\w+)',n); return m.group(1) if m else n[:30]
    seq=[(short(x['Kernel_Name']),(int(x['End_Timestamp'])-int(x['Start_Timestamp']))/1e3) for x in r]
    idx=[i for i,s in enumerate(seq) if s[0]=='bn_bwd_apply_kernel']
    last=idx[-19*5]
    tot=collections.defaultdict(float)
    for s in seq[last:idx[-1]+1]: tot[s[0]]+=s[1]
    print(d, {k:round(v/5,1) for k,v in sorted(tot.items()) if v/5>20})
