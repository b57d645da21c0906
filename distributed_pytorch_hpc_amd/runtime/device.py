"""GPU -> NUMA topology of the node and the per-rank CPU binding the launcher applies.

An 8x MI355X node hangs four GPUs off each CPU socket; a rank whose Python thread, data-loader workers and pinned
host buffers live on the other socket pays the inter-socket link on every host<->device copy and on every kernel
launch's doorbell.  The reference explicitly turns binding off (``mpiexec ... --cpu-bind none``,
scripts/02_fully_sharded_fsdp/run_fsdp.sh:64); here each rank is pinned to the cores of its GPU's NUMA node and
those cores are split between the ranks that share the node, so eight ranks never contend for one core set.

Only sysfs is read (no HIP call): the plan is computed in the launcher process and applied in the spawned child
before it execs Python (``preexec_fn``), i.e. before anything touches the GPU.

* ``gpus(sysfs)`` -- the node's AMD GPUs in PCI-bus order (the order HIP enumerates them), each with its NUMA node,
  the CPUs sysfs lists as local to it and whether this process can open its render node.  A container given a
  subset of the cards through device cgroups still sees every card in sysfs; HIP enumerates only the cards whose
  ``/dev/dri/renderD*`` node is present and openable, so those are the ones device ordinals (and
  *_VISIBLE_DEVICES) index.
* ``visible_indices(env)`` -- HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES as physical indices.
* ``plan(nproc, ...)`` -- rank r -> (physical GPU, NUMA node, disjoint CPU set, OMP thread count).

``DPH_SYSFS_ROOT`` points the reader at a fake tree (tests).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

AMD_VENDOR = "0x1002"
# PCI classes of AMD GPUs / accelerators: display (0x03xx) and processing accelerator (0x12xx, Instinct parts)
GPU_CLASS_PREFIXES = ("0x03", "0x12")


@dataclass
class GpuInfo:
    index: int                # physical index (PCI-bus order)
    bdf: str                  # PCI address, e.g. 0000:05:00.0
    numa_node: int            # -1 when the platform reports none
    local_cpus: list = field(default_factory=list)
    accessible: bool | None = None   # render node present and openable; None: unknown (no /dev/dri to check)


@dataclass
class RankBinding:
    rank: int
    gpu: int                  # physical GPU index
    numa_node: int
    cpus: list                # CPUs this rank is pinned to (empty: leave the affinity alone)
    omp_threads: int


def _root(sysfs: str | None) -> str:
    return sysfs or os.environ.get("DPH_SYSFS_ROOT", "/sys")


def _devroot(sysfs: str | None) -> str:
    """/dev for the real sysfs; a fake tree (tests) keeps its device nodes in a sibling ``dev`` directory."""
    root = _root(sysfs)
    return "/dev" if os.path.abspath(root) == "/sys" else os.path.join(os.path.dirname(os.path.abspath(root)), "dev")


def _render_access(dev: str, devroot: str) -> bool | None:
    """Whether one of the card's render nodes (``<device>/drm/renderD*``) exists and opens read-write under
    ``devroot/dri``; None when there is nothing to check against."""
    dri = os.path.join(devroot, "dri")
    try:
        nodes = [n for n in os.listdir(os.path.join(dev, "drm")) if n.startswith("renderD")]
    except OSError:
        return None
    if not nodes or not os.path.isdir(dri):
        return None
    return any(os.path.exists(os.path.join(dri, n)) and os.access(os.path.join(dri, n), os.R_OK | os.W_OK)
               for n in nodes)


def _read(path: str, default: str = "") -> str:
    try:
        with open(path) as fh:
            return fh.read().strip()
    except OSError:
        return default


def parse_cpulist(text: str) -> list:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11] (the kernel's cpulist format)."""
    out = []
    for part in text.replace("\n", ",").split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            lo, hi = part.split("-", 1)
            out.extend(range(int(lo), int(hi) + 1))
        else:
            out.append(int(part))
    return sorted(set(out))


def gpus(sysfs: str | None = None) -> list:
    """AMD GPUs found under <sysfs>/class/drm/card*/device, in PCI-bus order, de-duplicated by PCI address."""
    root = _root(sysfs)
    drm = os.path.join(root, "class", "drm")
    devroot = _devroot(sysfs)
    seen = {}
    try:
        cards = sorted(c for c in os.listdir(drm) if c.startswith("card") and c[4:].isdigit())
    except OSError:
        return []
    for c in cards:
        dev = os.path.join(drm, c, "device")
        if _read(os.path.join(dev, "vendor")) != AMD_VENDOR:
            continue
        if not _read(os.path.join(dev, "class")).startswith(GPU_CLASS_PREFIXES):
            continue
        bdf = os.path.basename(os.path.realpath(dev))
        if bdf in seen:
            continue
        try:
            node = int(_read(os.path.join(dev, "numa_node"), "-1"))
        except ValueError:
            node = -1
        cpus = parse_cpulist(_read(os.path.join(dev, "local_cpulist")))
        if not cpus and node >= 0:
            cpus = parse_cpulist(_read(os.path.join(root, "devices", "system", "node", f"node{node}", "cpulist")))
        seen[bdf] = (node, cpus, _render_access(dev, devroot))
    return [GpuInfo(i, bdf, n, c, a) for i, (bdf, (n, c, a)) in enumerate(sorted(seen.items()))]


def visible_indices(env: dict | None = None, n_physical: int | None = None) -> list | None:
    """Physical GPU indices the ranks' device ordinals map to, from the first *_VISIBLE_DEVICES variable set (HIP's
    precedence), or None when none is set.  UUID-style entries are not resolvable from sysfs: None."""
    env = os.environ if env is None else env
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        val = env.get(var)
        if val is None:
            continue
        try:
            idx = [int(v) for v in val.split(",") if v.strip() != ""]
        except ValueError:
            return None
        if n_physical is not None:
            idx = [i for i in idx if 0 <= i < n_physical]
        return idx
    return None


def plan(nproc: int, sysfs: str | None = None, env: dict | None = None, allowed: list | None = None,
         omp_threads: int = 0) -> list:
    """Per-rank binding: rank r drives device ordinal r (LOCAL_RANK), i.e. physical GPU visible[r]; it is pinned to
    its share of the CPUs local to that GPU (within the launcher's own affinity ``allowed``).  Ranks on one NUMA
    node split its CPUs into disjoint contiguous slices.  Without topology (no sysfs, no NUMA info) every rank keeps
    the full affinity and an even share of OMP threads."""
    if allowed is None:
        try:
            allowed = sorted(os.sched_getaffinity(0))
        except AttributeError:
            allowed = list(range(os.cpu_count() or 1))
    allowed_set = set(allowed)
    devs = gpus(sysfs)
    # the cards HIP can enumerate: those whose render node this process can open (all of them when unknown)
    usable = [g.index for g in devs if g.accessible is not False]
    vis = visible_indices(env, len(usable)) if usable else None
    phys = [usable[i] for i in vis] if vis is not None else usable
    out = []
    if not devs or len(phys) < nproc:
        share = max(1, len(allowed) // max(nproc, 1))
        return [RankBinding(r, r, -1, [], omp_threads or share) for r in range(nproc)]
    # group ranks by the CPU set local to their GPU (= NUMA node on every real platform)
    groups = {}
    for r in range(nproc):
        g = devs[phys[r]]
        local = [c for c in g.local_cpus if c in allowed_set]
        key = tuple(local)
        groups.setdefault(key, []).append(r)
    cpus_of = {}
    for key, ranks in groups.items():
        local = list(key)
        if not local:                    # GPU's node has none of our CPUs: leave those ranks unbound
            for r in ranks:
                cpus_of[r] = []
            continue
        k = len(ranks)
        per = len(local) // k
        for j, r in enumerate(ranks):
            if per == 0:                 # more ranks than local cores: share the node's cores
                cpus_of[r] = local
            else:
                cpus_of[r] = local[j * per:(j + 1) * per] if j < k - 1 else local[j * per:]
    for r in range(nproc):
        g = devs[phys[r]]
        cpus = cpus_of[r]
        threads = omp_threads or max(1, len(cpus) if cpus else len(allowed) // max(nproc, 1))
        out.append(RankBinding(r, g.index, g.numa_node, cpus, threads))
    return out


def describe(bindings: list) -> str:
    def rng(c):
        if not c:
            return "unbound"
        parts, start, prev = [], c[0], c[0]
        for x in c[1:] + [None]:
            if x is not None and x == prev + 1:
                prev = x
                continue
            parts.append(f"{start}-{prev}" if prev != start else f"{start}")
            if x is not None:
                start = prev = x
        return ",".join(parts)

    return "\n".join(f"rank {b.rank} -> GPU {b.gpu} -> NUMA {b.numa_node} -> CPUs {rng(b.cpus)} "
                     f"(OMP_NUM_THREADS={b.omp_threads})" for b in bindings)
