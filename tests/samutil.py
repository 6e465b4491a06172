"""SAM comparison helpers shared by the tests (grouping records per read)."""


def groups(data: bytes):
    """One group per input read: primary/unmapped record + its 0x800/0x100 records."""
    out = []
    for line in data.splitlines(keepends=True):
        f = line.split(b"\t")
        name, flag = f[0], int(f[1])
        if out and (flag & 0x900) and out[-1][0] == name:
            out[-1][1].append(line)
        else:
            out.append((name, [line]))
    return out


def compare(a: bytes, b: bytes):
    ga, gb = groups(a), groups(b)
    assert len(ga) == len(gb), (len(ga), len(gb))
    full = tax = mapped = 0
    for (na, la), (nb, lb) in zip(ga, gb):
        assert na == nb
        if la != lb:
            full += 1
        fa, fb = la[0].split(b"\t"), lb[0].split(b"\t")
        tax += fa[2] != fb[2]
        mapped += (int(fa[1]) & 4) != (int(fb[1]) & 4)
    return dict(reads=len(ga), full_mismatch=full, taxid_mismatch=tax, mapped_mismatch=mapped)


def ana_get_tid(recs, parent, max_tid):
    """meta_analysis' one-taxon-per-read rule (reference src/cly_mt.c:902-961) over the SAM
    records of one read: primary taxon, replaced by an equal-score later record's taxon
    when that taxon descends from it."""
    first = recs[0].split(b"\t")
    if first[2] == b"*":
        return 0

    def tid_score(f):
        t = int(f[2].split(b"|")[1])
        s = int(next(x for x in f if x.startswith(b"AS:i:"))[5:])
        return t, s

    tid, score = 0, 0
    t, s = tid_score(first)
    if t <= max_tid:
        tid, score = t, s
    for line in recs[1:]:
        if score == 0:
            break
        t, s = tid_score(line.split(b"\t"))
        if s != score or t > max_tid:
            continue
        p = t
        while True:
            if p == tid:
                tid = t
                break
            if p < 1 or p == 0xFFFFFFFF:
                break
            p = parent.get(p, 0xFFFFFFFF)
    return tid


def read_parents(nodes_dmp):
    """taxid -> parent taxid of an NCBI nodes.dmp (root's parent = 0xFFFFFFFF)."""
    parent = {}
    with open(nodes_dmp) as f:
        for line in f:
            a = [x.strip() for x in line.split("|")]
            t = int(a[0])
            parent[t] = int(a[1]) if t != 1 else 0xFFFFFFFF
    return parent
