"""Every hand-written kernel's PMC bytes land under the timing-registry id it
is launched with (verdict r4 #7: skip_bwd_c1_kernel had no entry in
tools/pmc_traffic.py, so skip_reduce_bwd read 0.51x, and the SE-over-BN
reduction was filed under bn_bwd_reduce, which read 1.45x).

For each MDE_LAUNCH / MDE_LAUNCH_MFMA site in csrc/*.hip: the K_* id ->
its name in timing.hip's table (enum order of common.h), and the launched
kernel's symbol (with the site's template arguments) -> pmc_traffic.NAMES;
the two must agree (a combined "a+b" key counts for both a and b).  CPU only.
"""
import importlib.util
import os
import re

from tests.conftest import REPO

CSRC = os.path.join(REPO, "monocular_depth_estimation_amd", "csrc")


def _registry():
    enum = open(os.path.join(CSRC, "common.h")).read()
    body = enum[enum.index("enum Kid"):enum.index("K_COUNT")]
    ids = re.findall(r"\b(K_\w+)", body)
    tim = open(os.path.join(CSRC, "timing.hip")).read()
    table = tim[tim.index("kNames[mde::K_COUNT]"):]
    table = table[:table.index("};")]
    names = re.findall(r'"(\w+)"', table)
    assert len(ids) == len(names), (len(ids), len(names))
    return dict(zip(ids, names))


def _pmc():
    spec = importlib.util.spec_from_file_location("pmc_traffic",
                                                  os.path.join(REPO, "tools", "pmc_traffic.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _sites():
    """(file, K id, kernel text incl. template args) of every launch with a literal id."""
    out = []
    for f in sorted(os.listdir(CSRC)):
        if not f.endswith(".hip"):
            continue
        text = open(os.path.join(CSRC, f)).read()
        for m in re.finditer(r"MDE_LAUNCH(?:_MFMA)?\(\s*(?:mde::|::mde::)?(K_\w+)\s*,", text):
            rest = text[m.end():m.end() + 400]
            k = re.search(r"\(?\s*(\w+_kernel(?:<[^>]*>)?)", rest)
            if k:
                out.append((f, m.group(1), k.group(1)))
    return out


_LITERAL = re.compile(r"^(\d+|true|false|float|T|uint8_t|int16_t|B|bf16|mde::bf16|k[A-Z]\w*)$")


def _literal_args(kern):
    """Template arguments that fix the symbol's leading arguments: numbers,
    bools, types, enumerators (kSum ...).  Sites whose leading arguments are
    macro / template parameters (A, CI, ...) are checked by the symbol test."""
    if "<" not in kern:
        return True
    args = [a.strip() for a in kern[kern.index("<") + 1:-1].split(",")]
    return all(_LITERAL.match(a) for a in args)


_ENUMS = {"kSum": "0", "kDot": "1", "kBnRelu": "2"}  # se.hip's se_partial_kernel modes


def test_every_launch_site_maps_to_its_registry_id():
    reg, pmc = _registry(), _pmc()
    sites = _sites()
    assert len(sites) > 60
    bad = []
    for f, kid, kern in sites:
        if not _literal_args(kern):
            continue
        for e, v in _ENUMS.items():
            kern = re.sub(rf"\b{e}\b", v, kern)
        want = reg[kid]
        got = pmc.registry_name(kern)
        if got is None or want not in got.split("+"):
            bad.append(f"{f}: {kern} launched as {kid} ({want}) but PMC-mapped to {got}")
    assert not bad, "\n".join(bad)


def test_variable_id_kernels_are_mapped():
    """Kernels launched with a runtime id (wino, convbf forward / data
    gradient) map to the combined key of both ids."""
    pmc = _pmc()
    assert pmc.registry_name("wino_f23_kernel<64, 8, false>") == "wino_fwd+wino_dgrad"
    assert pmc.registry_name("convbf_fwd_kernel<3, 0, 2, 2, false, 420>") == \
        "convbf_fwd_bf16+convbf_dgrad_bf16"


def test_profiled_hand_kernels_are_all_mapped():
    """Every hand-written kernel symbol in the committed rocprofv3 kernel
    statistics maps to some registry id (nothing silently dropped)."""
    import csv
    import glob
    pmc = _pmc()
    ours = set()
    for f in os.listdir(CSRC):
        if f.endswith(".hip"):
            ours |= set(re.findall(r"\b(\w+_kernel)\s*\(", open(os.path.join(CSRC, f)).read()))
    ours.discard("graph_fill_kernel")  # the captured-memset repair (csrc/graph.hip): no registry id
    seen, bad = 0, []
    for path in glob.glob(os.path.join(REPO, "profiles", "r0[45]_*kernel_stats.csv")):
        with open(path) as fh:
            for row in csv.DictReader(fh):
                sym = row.get("Name") or row.get("KernelName") or ""
                m = re.search(r"(\w+_kernel)\b", sym)
                base = m.group(1) if m else ""
                if base in ours:
                    seen += 1
                    if pmc.registry_name(sym) is None:
                        bad.append(f"{os.path.basename(path)}: {sym[:120]}")
    assert seen > 50, seen
    assert not bad, "\n".join(sorted(set(bad)))
