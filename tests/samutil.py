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
