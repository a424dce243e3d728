"""CPU restatement of record decoding for parity tests (test infrastructure; never the
product path).

Follows the BAM record layout htsjdk's BAMRecordCodec.decode reads
(check/.../iterator/RecordStream.scala:16-41 drives it over the record chain): the chain
from the first record after the header (next = start + 4 + block_size), the fixed
fields, read name, CIGAR, 4-bit bases, qualities and raw tags.  `sam_line` renders a
record like htsjdk's SAMRecord.getSAMString; it is written independently of the
package's renderer and pinned against the reference's test_bams/2.sam.
"""
import struct

import numpy as np

SEQ = "=ACMGRSVTWYHKDBN"
OPS = "MIDNSHP=X"


def bam_refs(flat):
    """(reference names, flat offset of the first record) from the BAM header."""
    b = bytes(flat[:1 << 20])
    assert b[:4] == b"BAM\1"
    l_text = struct.unpack_from("<i", b, 4)[0]
    p = 8 + l_text
    n_ref = struct.unpack_from("<i", b, p)[0]
    p += 4
    names = []
    for _ in range(n_ref):
        ln = struct.unpack_from("<i", b, p)[0]
        names.append(b[p + 4:p + 4 + ln - 1].decode("ascii"))
        p += 4 + ln + 4
    return names, p


def record_starts(flat, first, end):
    out, r = [], first
    while r < end and r + 4 <= len(flat):
        out.append(r)
        r += 4 + struct.unpack_from("<i", flat, r)[0]
    return out


def decode(flat, starts):
    """Columns in the layout of the package's Reads (numpy arrays)."""
    f = bytes(flat)
    cols = {k: [] for k in ("flat", "ref_id", "pos", "next_ref_id", "next_pos", "tlen", "flag", "bin", "mapq")}
    names, cigar, seq, qual, aux = bytearray(), [], bytearray(), bytearray(), bytearray()
    offs = {k: [0] for k in ("name_off", "cigar_off", "seq_off", "aux_off")}
    for p in starts:
        bsz, ref, pos, bmn, fnc, lseq, nref, npos, tlen = struct.unpack_from("<iiiIIiiii", f, p)
        lname, ncig = bmn & 0xff, fnc & 0xffff
        cols["flat"].append(p)
        cols["ref_id"].append(ref)
        cols["pos"].append(pos)
        cols["next_ref_id"].append(nref)
        cols["next_pos"].append(npos)
        cols["tlen"].append(tlen)
        cols["flag"].append(fnc >> 16)
        cols["bin"].append(bmn >> 16)
        cols["mapq"].append((bmn >> 8) & 0xff)
        q = p + 36
        names += f[q:q + lname]
        q += lname
        cigar.extend(struct.unpack_from("<%dI" % ncig, f, q))
        q += 4 * ncig
        for k in range(lseq):
            byte = f[q + k // 2]
            seq.append(ord(SEQ[(byte & 15) if k & 1 else byte >> 4]))
        q += (lseq + 1) // 2
        qual += f[q:q + lseq]
        q += lseq
        aux += f[q:p + 4 + bsz]
        offs["name_off"].append(len(names))
        offs["cigar_off"].append(len(cigar))
        offs["seq_off"].append(len(seq))
        offs["aux_off"].append(len(aux))
    dt = {"flat": np.uint64, "ref_id": np.int32, "pos": np.int32, "next_ref_id": np.int32,
          "next_pos": np.int32, "tlen": np.int32, "flag": np.uint16, "bin": np.uint16, "mapq": np.uint8}
    out = {k: np.asarray(v, dtype=dt[k]) for k, v in cols.items()}
    out.update({k: np.asarray(v, dtype=np.uint64) for k, v in offs.items()})
    out["names"] = np.frombuffer(bytes(names), np.uint8)
    out["cigar"] = np.asarray(cigar, np.uint32)
    out["seq"] = np.frombuffer(bytes(seq), np.uint8)
    out["qual"] = np.frombuffer(bytes(qual), np.uint8)
    out["aux"] = np.frombuffer(bytes(aux), np.uint8)
    return out


def _tag_strings(b):
    fmts = {"c": "b", "C": "B", "s": "h", "S": "H", "i": "i", "I": "I"}
    out, i = [], 0
    while i < len(b):
        tag, t = b[i:i + 2].decode(), chr(b[i + 2])
        i += 3
        if t == "A":
            out.append(f"{tag}:A:{chr(b[i])}")
            i += 1
        elif t in fmts:
            v = struct.unpack_from("<" + fmts[t], b, i)[0]
            out.append(f"{tag}:i:{v}")
            i += struct.calcsize(fmts[t])
        elif t in "ZH":
            j = b.index(0, i)
            out.append(f"{tag}:{t}:{b[i:j].decode('latin-1')}")
            i = j + 1
        else:
            raise NotImplementedError(t)  # (f / B: not present in the pinned fixtures)
    return out


def sam_line(cols, i, refs):
    c = cols
    s = lambda k: int(c[k][i])  # noqa: E731
    n0, n1 = s("name_off"), int(c["name_off"][i + 1])
    name = bytes(c["names"][n0:n1 - 1]).decode()
    ref, nref = s("ref_id"), s("next_ref_id")
    cig = c["cigar"][s("cigar_off"):int(c["cigar_off"][i + 1])]
    sq = bytes(c["seq"][s("seq_off"):int(c["seq_off"][i + 1])]).decode()
    ql = c["qual"][s("seq_off"):int(c["seq_off"][i + 1])]
    return "\t".join([
        name, str(s("flag")), refs[ref] if ref >= 0 else "*", str(s("pos") + 1), str(s("mapq")),
        "".join(f"{int(v) >> 4}{OPS[int(v) & 15]}" for v in cig) or "*",
        "*" if nref < 0 else "=" if nref == ref else refs[nref], str(s("next_pos") + 1), str(s("tlen")),
        sq or "*", "*" if len(ql) == 0 or ql[0] == 0xFF else "".join(chr(int(x) + 33) for x in ql),
    ] + _tag_strings(bytes(c["aux"][s("aux_off"):int(c["aux_off"][i + 1])])))


REF_OPS = (0, 2, 3, 7, 8)  # M D N = X consume the reference


def region(cols, i):
    """CanLoadBam.region (load/.../CanLoadBam.scala:446-454) as (ref_idx, begin, end) or
    None: no contig for refID -1; htsjdk getAlignmentEnd is 0 for an unmapped read and
    alignmentStart + referenceLength - 1 otherwise; Region(contig, start - 1, end)."""
    ref = int(cols["ref_id"][i])
    if ref < 0:
        return None
    start = int(cols["pos"][i]) + 1
    if cols["flag"][i] & 4:
        end = 0
    else:
        ops = cols["cigar"][cols["cigar_off"][i]:cols["cigar_off"][i + 1]]
        end = start + sum(int(o) >> 4 for o in ops if (int(o) & 15) in REF_OPS) - 1
    return ref, start - 1, end


def region_kept(cols, i, loci_by_ref):
    """LociSet.intersects(region): some half-open range [a, b) of the contig with
    max(a, begin) < min(b, end) (a non-empty Guava range intersection)."""
    r = region(cols, i)
    if r is None:
        return False
    ref, b, e = r
    return any(max(a, b) < min(z, e) for a, z in loci_by_ref.get(ref, ()))


def interval_records(flat, chunk_flats, loci_by_ref):
    """loadBamIntervals' record loop (CanLoadBam.scala:132-152), one chunk after the
    other: the chain from the chunk start while the start is < the chunk end, kept when
    the region overlaps.  Returns (decoded columns of the kept records, per-chunk counts)."""
    starts, per = [], []
    for a, e in chunk_flats:
        cs = record_starts(flat, a, min(e, len(flat)))
        cols = decode(flat, cs)
        kept = [cs[i] for i in range(len(cs)) if region_kept(cols, i, loci_by_ref)]
        starts += kept
        per.append(len(kept))
    return decode(flat, starts), per
