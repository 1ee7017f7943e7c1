"""Kernel names of rocprofv3 traces -> the variants and families the profile tools report.

k_closest / k_shadow are instantiated <kPacket, kCount, kMesh> (trace.hip): the counting
instantiations (kCount true: bench.py's solo pass makes one counting call for the work counts,
the roofline times the other) are dropped; the rest are named by their remaining arguments
(k_shadow<true, true> = packets, with the mesh search).  k_fused is <kPacket, kMesh>."""
import re

_RE = re.compile(r"(k_[a-z0-9_]+)(?:<([^>]*)>)?\(")


def parse(name):
    """(family, variant) of a kernel name, or (None, None) for a counting instantiation or a
    name that is not one of the path's kernels."""
    m = _RE.search(name)
    if not m:
        return None, None
    fam = m.group(1)
    args = [a.strip() for a in (m.group(2) or "").split(",") if a.strip()]
    if fam in ("k_closest", "k_shadow") and len(args) >= 2:
        if args[1] == "true":
            return None, None
        args = [args[0]] + args[2:]
    return fam, fam + ("<" + ", ".join(args) + ">" if args else "")
