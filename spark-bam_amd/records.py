"""Columnar BAM records decoded on the GPU (sbh_records_scan / sbh_records_fetch) and
their SAM text.

The reference hands htsjdk SAMRecords out of RecordStream / CanLoadBam.loadReads
(check/.../iterator/RecordStream.scala:16-41, load/.../CanLoadBam.scala:244-264); here a
batch is a set of numpy columns filled by libsparkbam_hip.so.  `sam_line` renders one
record the way htsjdk's SAMRecord.getSAMString does (the format of the reference's
test_bams/*.sam files), for inspection and tests; the decode itself is the GPU's.
"""
import struct

import numpy as np

CIGAR_OPS = "MIDNSHP=X"

# The columns sbh_records_fetch fills (sbh_records_out field order): name -> (dtype, length
# from (n, name_bytes, cigar_ops, bases, aux_bytes)).  Offset columns hold n + 1 entries.
RECORD_COLUMNS = (
    ("flat", np.uint64, lambda n, nm, cg, bs, ax: n), ("ref_id", np.int32, lambda n, *_: n),
    ("pos", np.int32, lambda n, *_: n), ("next_ref_id", np.int32, lambda n, *_: n),
    ("next_pos", np.int32, lambda n, *_: n), ("tlen", np.int32, lambda n, *_: n),
    ("flag", np.uint16, lambda n, *_: n), ("bin", np.uint16, lambda n, *_: n),
    ("mapq", np.uint8, lambda n, *_: n), ("name_off", np.uint64, lambda n, *_: n + 1),
    ("cigar_off", np.uint64, lambda n, *_: n + 1), ("seq_off", np.uint64, lambda n, *_: n + 1),
    ("aux_off", np.uint64, lambda n, *_: n + 1), ("names", np.uint8, lambda n, nm, cg, bs, ax: nm),
    ("cigar", np.uint32, lambda n, nm, cg, bs, ax: cg), ("seq", np.uint8, lambda n, nm, cg, bs, ax: bs),
    ("qual", np.uint8, lambda n, nm, cg, bs, ax: bs), ("aux", np.uint8, lambda n, nm, cg, bs, ax: ax),
)


def record_columns(n=0, name_bytes=0, cigar_ops=0, bases=0, aux_bytes=0):
    """Uninitialised columns for n records (offset columns zeroed when n == 0, so an empty
    batch has the same schema as a full one)."""
    z = (n, name_bytes, cigar_ops, bases, aux_bytes)
    cols = {k: (np.zeros if n == 0 else np.empty)(f(*z), dt) for k, dt, f in RECORD_COLUMNS}
    return cols
_B_FMT = {"c": "b", "C": "B", "s": "h", "S": "H", "i": "i", "I": "I", "f": "f"}


def _java_float(x):
    """java.lang.Float.toString for the finite values a BAM 'f' tag holds."""
    if x != x:
        return "NaN"
    if x in (float("inf"), float("-inf")):
        return "Infinity" if x > 0 else "-Infinity"
    for p in range(1, 10):  # shortest digits that read back as the same float32
        s = "%.*g" % (p, x)
        if np.float32(float(s)) == np.float32(x):
            break
    if "e" in s or "E" in s:
        m, e = s.split("e")
        if "." not in m:
            m += ".0"
        return "%sE%d" % (m, int(e))
    return s if "." in s else s + ".0"


def tags_text(aux):
    """The SAM text of a record's raw tag bytes (TAG:TYPE:VALUE, tab separated)."""
    out, i, b = [], 0, bytes(aux)
    while i + 3 <= len(b):
        tag, t = b[i:i + 2].decode("ascii"), chr(b[i + 2])
        i += 3
        if t == "A":
            out.append("%s:A:%s" % (tag, chr(b[i])))
            i += 1
        elif t in "cCsSiI":
            fmt = _B_FMT[t]
            n = struct.calcsize(fmt)
            out.append("%s:i:%d" % (tag, struct.unpack_from("<" + fmt, b, i)[0]))
            i += n
        elif t == "f":
            out.append("%s:f:%s" % (tag, _java_float(struct.unpack_from("<f", b, i)[0])))
            i += 4
        elif t in "ZH":
            j = b.index(b"\0", i)
            out.append("%s:%s:%s" % (tag, t, b[i:j].decode("latin-1")))
            i = j + 1
        elif t == "B":
            sub, n = chr(b[i]), struct.unpack_from("<i", b, i + 1)[0]
            i += 5
            fmt = _B_FMT[sub]
            vals = struct.unpack_from("<%d%s" % (n, fmt), b, i)
            i += n * struct.calcsize(fmt)
            txt = ",".join(_java_float(v) if sub == "f" else str(v) for v in vals)
            out.append("%s:B:%s%s" % (tag, sub, "," + txt if n else ""))
        else:
            raise ValueError("unknown tag type %r" % t)
    return out


class Reads:
    """A decoded batch: fixed fields as arrays, variable-length fields packed."""

    def __init__(self, cols, ref_names):
        self.cols = cols
        self.ref_names = list(ref_names)
        self.n = int(cols["flat"].size)

    def __len__(self):
        return self.n

    OFFSETS = {"name_off": "names", "cigar_off": "cigar", "seq_off": "seq", "aux_off": "aux"}

    @classmethod
    def concat(cls, batches, ref_names):
        """One batch of the records of several, in order (windowed loadReads, api.iter_reads)."""
        batches = [b for b in batches if b.n]
        if not batches:
            cols = record_columns()
            cols["vpos"] = np.empty(0, np.uint64)
            return cls(cols, ref_names)
        cols = {}
        for k in batches[0].cols:
            if k in cls.OFFSETS:
                parts, base = [], 0
                for b in batches:
                    o = b.cols[k]
                    parts.append(o[:-1] + base)
                    base += int(o[-1])
                parts.append(np.asarray([base], dtype=batches[0].cols[k].dtype))
                cols[k] = np.concatenate(parts)
            else:
                cols[k] = np.concatenate([b.cols[k] for b in batches])
        return cls(cols, ref_names)

    def _slice(self, name, off, i):
        o = self.cols[off]
        return self.cols[name][int(o[i]):int(o[i + 1])]

    def name(self, i):
        return bytes(self._slice("names", "name_off", i)).split(b"\0", 1)[0].decode("latin-1")

    def cigar(self, i):
        ops = self._slice("cigar", "cigar_off", i)
        return "".join("%d%s" % (int(v) >> 4, CIGAR_OPS[int(v) & 15]) for v in ops) or "*"

    def seq(self, i):
        return bytes(self._slice("seq", "seq_off", i)).decode("ascii") or "*"

    def qual(self, i):
        q = self._slice("qual", "seq_off", i)
        if q.size == 0 or q[0] == 0xFF:
            return "*"
        return bytes((q + 33).astype(np.uint8)).decode("ascii")

    def tags(self, i):
        return tags_text(self._slice("aux", "aux_off", i))

    def sam_line(self, i):
        c = self.cols
        ref, nref = int(c["ref_id"][i]), int(c["next_ref_id"][i])
        rname = self.ref_names[ref] if 0 <= ref < len(self.ref_names) else "*"
        if nref < 0:
            rnext = "*"
        elif nref == ref:
            rnext = "="
        else:
            rnext = self.ref_names[nref] if nref < len(self.ref_names) else "*"
        fields = [self.name(i), str(int(c["flag"][i])), rname, str(int(c["pos"][i]) + 1),
                  str(int(c["mapq"][i])), self.cigar(i), rnext, str(int(c["next_pos"][i]) + 1),
                  str(int(c["tlen"][i])), self.seq(i), self.qual(i)]
        return "\t".join(fields + self.tags(i))

    def sam_lines(self):
        return [self.sam_line(i) for i in range(self.n)]
