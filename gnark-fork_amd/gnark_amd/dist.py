"""Multi-GPU MSM sharding over RCCL (one process per GPU, torch.distributed).

The MSM point set shards naturally: rank k keeps the contiguous slice
shard_range(n, k, world) of every key array resident in its own HBM, runs
gg_msm on it and returns a Jacobian partial.  Partials are all-gathered (96 B
per G1 MSM, 192 B per G2) and added on every rank with gg_g1/g2_jac_add --
RCCL has no elliptic-curve reduction op, so this is gather + add, not reduce.
No other data crosses xGMI on the MSM path.
"""
from __future__ import annotations

from . import msm

_JAC = {msm.G1: 96, msm.G2: 192}


def shard_range(n: int, rank: int, world: int):
    """Contiguous, balanced slice [lo, hi) of n points owned by `rank`."""
    lo = n * rank // world
    hi = n * (rank + 1) // world
    return lo, hi


def combine_partials(group: int, partials) -> bytes:
    """Sum of Jacobian partials (bytes) with the library's exact group law."""
    acc = partials[0]
    for p in partials[1:]:
        acc = msm.jac_add(group, acc, p)
    return acc


def allgather_partial(group: int, jac: bytes, device=None) -> bytes:
    """All-gather every rank's partial and return the (identical) sum on all ranks."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    if world == 1:
        return jac
    t = torch.frombuffer(bytearray(jac), dtype=torch.uint8)
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return combine_partials(group, [bytes(p.cpu().numpy()) for p in parts])


def group_devices(local_device: int, device=None) -> list:
    """The GPU id of every rank of the process group, in rank order (all-gather)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [int(local_device)]
    t = torch.tensor([int(local_device)], dtype=torch.int64)
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [int(p.item()) for p in parts]


def broadcast_bytes(data, nbytes: int, src: int = 0, device=None) -> bytes:
    """`data` (nbytes, significant on rank `src`) on every rank."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return bytes(data)
    if dist.get_rank() == src:
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    else:
        t = torch.zeros(nbytes, dtype=torch.uint8)
    if device is not None:
        t = t.to(device)
    dist.broadcast(t, src)
    return bytes(t.cpu().numpy())


# ---------------------------------------------------------------- failures
# gnark ends a proof at the first error of any of its concurrent tasks: the
# Groth16 prover's channels (backend/groth16/bn254/prove.go:198-209) and the
# PlonK prover's errgroup (backend/plonk/bls12-381/prove.go:132-173).  Over a
# process group the same has to hold across ranks: a rank whose part of the
# proof fails must not leave its peers blocked in the next collective until the
# group's timeout.  RankGuard gives every collective step of a proof a status
# step before it (an all-gather of one status record per rank), so every rank
# learns of a failure at the same step and raises.

STATUS_BYTES = 256  # per rank: [0] = 0 ok / 1 failed, then the error text (utf-8)


def _status_record(ok: bool, msg: str = "") -> bytearray:
    rec = bytearray(STATUS_BYTES)
    if not ok:
        rec[0] = 1
        m = msg.encode("utf-8", "replace")[:STATUS_BYTES - 1]
        rec[1:1 + len(m)] = m
    return rec


def _status_text(rec: bytes) -> str:
    return bytes(rec[1:]).split(b"\0", 1)[0].decode("utf-8", "replace")


class RankFailure(RuntimeError):
    """Another rank's part of the proof failed (errgroup semantics across ranks):
    `failed` maps each failing rank to its error text."""

    def __init__(self, failed: dict, stage: str = ""):
        self.failed = dict(failed)
        where = f" at {stage}" if stage else ""
        parts = "; ".join(f"rank {r}: {m or 'error'}" for r, m in sorted(self.failed.items()))
        super().__init__(f"proof aborted{where}: {parts}")


class RankGuard:
    """Status steps of one distributed proof.  check() before every collective
    of the proof (and before the final gather): returns if every rank is still
    fine, else raises RankFailure on every rank.  A rank whose own work raised
    calls fail(err) once -- it takes part in the status step its peers wait in,
    so they raise instead of waiting -- and then re-raises its error.
    device: where the status tensor lives (the RCCL device under "nccl")."""

    def __init__(self, device=None, stage: str = "proof"):
        self.device = device
        self.stage = stage
        self.failed = None  # dict of the agreed failure, once a status step saw one

    def _exchange(self, rec: bytearray) -> list:
        import torch
        import torch.distributed as dist
        if not dist.is_initialized() or dist.get_world_size() == 1:
            return [bytes(rec)]
        t = torch.frombuffer(rec, dtype=torch.uint8)
        if self.device is not None:
            t = t.to(self.device)
        parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, t)
        return [bytes(p.cpu().numpy()) for p in parts]

    def check(self, what: str = ""):
        if self.failed is not None:
            raise RankFailure(self.failed, what or self.stage)
        recs = self._exchange(_status_record(True))
        bad = {r: _status_text(x) for r, x in enumerate(recs) if x[0]}
        if bad:
            self.failed = bad
            raise RankFailure(bad, what or self.stage)

    def fail(self, err: BaseException):
        """this rank failed: join the status step its peers are in (once)"""
        if self.failed is not None:
            return
        import torch.distributed as dist
        me = dist.get_rank() if dist.is_initialized() else 0
        recs = self._exchange(_status_record(False, f"{type(err).__name__}: {err}"))
        self.failed = {r: _status_text(x) for r, x in enumerate(recs) if x[0]}
        self.failed.setdefault(me, str(err))

    def run(self, fn, *args, **kw):
        """fn(*args) with errgroup semantics: a failure on this rank is announced
        to the peers' next status step and re-raised; a peer's failure seen by a
        status step inside fn (e.g. in an exchange callback, where it surfaces as
        a library error) is raised as RankFailure."""
        try:
            return fn(*args, **kw)
        except RankFailure:
            raise
        except BaseException as e:
            if self.failed is not None:  # a status step inside fn saw a peer's failure
                raise RankFailure(self.failed, self.stage) from e
            self.fail(e)
            raise


def broadcast_status(ok: bool, msg: str = "", payload: bytes = b"", nbytes: int = 0, src: int = 0,
                     device=None, stage: str = "") -> bytes:
    """rank `src`'s status and payload (nbytes) on every rank: one broadcast.
    Raises RankFailure on the other ranks when src failed (src itself re-raises
    its own error); returns the payload."""
    import torch.distributed as dist
    rec = _status_record(ok, msg)
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return bytes(payload)
    me = dist.get_rank()
    if me == src:
        body = bytes(payload) if ok else b""
        assert not ok or len(body) == nbytes, "payload must be nbytes long"
        data = bytes(rec) + body.ljust(nbytes, b"\0")
    else:
        data = bytes(STATUS_BYTES + nbytes)
    got = broadcast_bytes(data, STATUS_BYTES + nbytes, src, device)
    if got[0] and me != src:
        raise RankFailure({src: _status_text(got[:STATUS_BYTES])}, stage)
    return got[STATUS_BYTES:]


# ------------------------------------------------------ leader-key devices
def device_identity(device: int):
    """A GPU's identity as this process sees it (PCI domain:bus:device and UUID),
    or None if this process cannot open that device id."""
    import torch
    try:
        if device < 0 or device >= torch.cuda.device_count():
            return None
        p = torch.cuda.get_device_properties(device)
    except Exception:  # no HIP device / driver: nothing visible
        return None
    return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x} {p.uuid}"


def group_identities(ident, device=None) -> list:
    """every rank's identity string (device_identity of its GPU), in rank order"""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [ident]
    rec = bytearray(128)
    b = (ident or "").encode()[:127]
    rec[:len(b)] = b
    t = torch.frombuffer(rec, dtype=torch.uint8)
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    out = []
    for p in parts:
        s = bytes(p.cpu().numpy()).split(b"\0", 1)[0].decode()
        out.append(s or None)
    return out


def check_leader_devices(devices, idents, view, backend=None) -> list:
    """Problems with a leader key over `devices` (rank r's GPU id, as rank r
    numbers it) whose identities the ranks reported as `idents`; view(d) is the
    identity rank 0 sees behind id d (None: not visible).  The leader opens every
    rank's GPU under that rank's id, so each id must name the same GPU on rank 0;
    under RCCL no two ranks may share a GPU (gloo rehearsals may)."""
    probs = []
    for r, (d, ident) in enumerate(zip(devices, idents)):
        v = view(d)
        if v is None:
            probs.append(f"rank {r}'s GPU {d} is not visible to rank 0 (a launcher that gives each rank its own "
                         f"HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES hides it; the leader key needs every GPU "
                         f"visible to rank 0)")
        elif ident is not None and v != ident:
            probs.append(f"rank {r}'s GPU {d} is {ident}, but rank 0's GPU {d} is {v} (the ranks number the GPUs "
                         f"differently: per-rank HIP_VISIBLE_DEVICES?)")
    if backend == "nccl":
        seen = {}
        for r, ident in enumerate(idents):
            key = ident if ident is not None else f"id {devices[r]}"
            if key in seen:
                probs.append(f"ranks {seen[key]} and {r} share GPU {key} under RCCL (one rank per GPU)")
            else:
                seen[key] = r
    return probs
