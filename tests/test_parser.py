"""The FASTQ/FASTA parser of the read_classify pipeline (desamba-so_amd/csrc/fastq.c), on the CPU.

The parser is a resumable emulation of the reference's kseq_read inside its 3-worker
kt_pipeline (reference src/lib/utils.c:839-977, src/cly_mt.c:29-43, 361-381); single-line
FASTQ records are taken as views of the input by a memchr fast path.  Pinned here:
  * fast path == byte-level emulation, whole input and in streaming batches of any size, on
    inputs built to hit every branch kseq has (FASTA records and the every-other-record drop,
    multi-line sequences and qualities, blank lines, CRLF, NUL bytes, garbage between records,
    malformed records ending a kt batch, truncated input, 5000-read / 10 Mbp batch limits);
  * the emulation == the committed golden inputs' record counts (the reference's SAM has one
    group per parsed read).
"""
import os
import random

import pytest

from conftest import golden
from samutil import groups


def recs(pyd, data, slow=False, batch=0):
    return pyd.parse_dump(data, slow=slow, batch_reads=batch)


def fq(name, seq, qual=None, plus=b"+"):
    return b"@" + name + b"\n" + seq + b"\n" + plus + b"\n" + (qual if qual is not None else b"I" * len(seq)) + b"\n"


def _random_input(rng: random.Random) -> bytes:
    parts = []
    for i in range(rng.randint(1, 400)):
        k = rng.random()
        seq = bytes(rng.choice(b"ACGTN") for _ in range(rng.choice([0, 1, 5, 40, 151, 1000])))
        name = b"r%d" % i + rng.choice([b"", b" comment x", b"\tc", b"\r"])
        if k < 0.70:
            parts.append(fq(name, seq))
        elif k < 0.75:  # FASTA record
            parts.append(b">" + name + b"\n" + seq + b"\n")
        elif k < 0.78:  # multi-line sequence + quality
            h = len(seq) // 2
            parts.append(b"@" + name + b"\n" + seq[:h] + b"\n" + seq[h:] + b"\n+\n" + b"J" * h + b"\n"
                         + b"J" * (len(seq) - h) + b"\n")
        elif k < 0.80:  # quality shorter / longer: malformed, ends the kt batch
            parts.append(fq(name, seq, b"I" * max(0, len(seq) + rng.choice([-1, 1]))))
        elif k < 0.82:  # blank line inside the sequence
            parts.append(b"@" + name + b"\n\n" + seq + b"\n+\n" + b"I" * (len(seq) + 1) + b"\n")
        elif k < 0.84:  # CRLF
            parts.append(b"@" + name + b"\r\n" + seq + b"\r\n+\r\n" + b"I" * len(seq) + b"\r\n")
        elif k < 0.86:  # garbage before the header
            parts.append(b"xx yy\n" + fq(name, seq))
        elif k < 0.88:  # NUL bytes in name / sequence
            parts.append(fq(name + b"\0z", seq[:3] + b"\0" + seq[3:]))
        elif k < 0.90:  # quality line starting with '@' and a '+name' separator line
            parts.append(fq(name, seq, b"@" * len(seq), plus=b"+" + name))
        elif k < 0.92:  # header only at the end / '>' inside quality
            parts.append(fq(name, seq, (b">" + b"I" * len(seq))[: len(seq)]))
        else:
            parts.append(fq(name, seq))
    data = b"".join(parts)
    cut = rng.random()
    if cut < 0.1:
        data = data[: rng.randint(0, len(data))]  # truncated input
    elif cut < 0.15:
        data = data + b"\0"  # main_test_2.c's input_n = fsize + 1
    elif cut < 0.2:
        data = data.rstrip(b"\n")
    return data


@pytest.mark.parametrize("seed", range(60))
def test_fast_path_equals_byte_level_emulation_on_adversarial_inputs(pyd, seed):
    rng = random.Random(seed)
    data = _random_input(rng)
    want = recs(pyd, data, slow=True)
    assert recs(pyd, data) == want
    for b in (1, 7, 1000):
        assert recs(pyd, data, batch=b) == want


def test_batch_limits_5000_reads_and_10_mbp():
    """More than 5000 short reads and reads summing past 10 Mbp cross kt_pipeline batch
    boundaries (cly_mt.c:22-23,33); FASTA records there exercise each worker's own slots."""
    import importlib
    pyd = importlib.import_module("conftest").load_pydesamba()
    parts = [fq(b"s%d" % i, b"ACGT" * 10) for i in range(12000)]
    parts += [fq(b"l%d" % i, b"A" * 900000) for i in range(25)]
    parts += [b">f%d\nACGTACGT\n" % i for i in range(30)]
    parts += [fq(b"t%d" % i, b"C" * 50) for i in range(6000)]
    data = b"".join(parts)
    want = recs(pyd, data, slow=True)
    assert recs(pyd, data) == want
    assert recs(pyd, data, batch=4096) == want
    # the FASTA records after the FASTQ ones: every other one is dropped (slot last_char)
    names = [l.split(b"\t", 1)[0] for l in want.splitlines()]
    assert names.count(b"s0") == 1 and len([n for n in names if n.startswith(b"f")]) < 30


@pytest.mark.parametrize("name", ["mixed", "ont", "illumina", "ont_long"])
def test_golden_inputs_parse_to_the_references_read_count(pyd, name):
    data = golden(name + ".fq")
    out = recs(pyd, data)
    assert out == recs(pyd, data, slow=True)
    assert len(out.splitlines()) == len(groups(golden(name + ".herm.sam")))
