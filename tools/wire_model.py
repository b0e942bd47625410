"""Modeled interconnect for one-GPU rehearsals of the row-partitioned step
(development and tests; not product code).

gloo -- the only backend the CPU tests and a one-GPU box can run several ranks
on -- stages every collective through host memory and completes it before the
call returns (`distributed.a2a` / `ag` hand back an already finished `_Done`).
So the `async_op=True` + `work.wait()` paths of `spgemm_new_amd/distributed.py`
never had a collective in flight while kernels ran (missing #1).
This module gives them one, with RCCL's stream semantics:

* the collective is ordered after the work already queued on the caller's
  current stream (an event recorded there, waited on by a side stream);
* on the side stream a spin kernel stands for the wire -- bytes / modeled
  per-rank rate -- and then the delivery copy runs;
* the input and output tensors are recorded on the side stream (as
  ProcessGroupNCCL does), so the caching allocator does not hand their memory to
  other work before the collective is done;
* ``wait()`` makes the caller's current stream wait for the side stream's done
  event(s); the host never blocks.

``Wire``: one rank alone on the GPU (timing: `tools/exp_rank_step.py --wire`).
``ThreadFabric``: all ranks of a world as threads of one process, each with its
own current stream and side stream, every collective a real exchange between
their tensors (correctness under concurrency: `tests/test_wire_overlap.py`).

Limits: the ranks must call the collectives from their own threads, so torch
autograd (whose backward runs on one engine thread per device) cannot drive a
partitioned backward here -- the explicit forward / backward calls can; and the
spin kernel is one wave, where RCCL's kernels hold several CUs.
"""
from __future__ import annotations

import threading

import torch

_CYCLES_PER_US = {}


def cycles_per_us(device) -> float:
    """Calibrate torch.cuda._sleep (a spin on the shader clock counter) once."""
    device = torch.device(device)
    if device not in _CYCLES_PER_US:
        n = 2_000_000
        torch.cuda._sleep(n)          # warm-up (first launch)
        torch.cuda.synchronize(device)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        torch.cuda._sleep(n)
        b.record()
        b.synchronize()
        _CYCLES_PER_US[device] = n / (a.elapsed_time(b) * 1e3)
    return _CYCLES_PER_US[device]


def spin_us(us: float, device) -> None:
    """A kernel that occupies the current stream for about `us` microseconds
    (one workgroup: it takes no bandwidth and almost no compute)."""
    if us > 0:
        torch.cuda._sleep(max(1, int(us * cycles_per_us(device))))


class Work:
    """RCCL-like work handle: wait() orders the caller's current stream after
    the collective (no host block)."""

    def __init__(self, events):
        self.events = events
        self.waited = False

    def wait(self):
        st = torch.cuda.current_stream()
        for ev in self.events:
            st.wait_event(ev)
        self.waited = True
        return None


class NoWaitWork(Work):
    """A handle whose wait() does nothing -- the negative control that proves a
    test would see a missing wait (the delivery lands after the consumer ran)."""

    def wait(self):
        self.waited = True
        return None


def _wire_us(nbytes: int, rate_GBs: float | None, latency_us: float) -> float:
    if rate_GBs is None:
        return 0.0
    return latency_us + nbytes / (rate_GBs * 1e3)


class Wire:
    """One rank's modeled link: ``issue(nbytes, deliver, tensors)`` runs
    `deliver()` (which writes the received bytes) on a side stream, after the
    caller's queued work and a spin of nbytes / rate (+ latency)."""

    def __init__(self, device, rate_GBs: float | None = None, latency_us: float = 10.0,
                 no_wait: bool = False):
        self.device = torch.device(device)
        self.side = torch.cuda.Stream(self.device)
        self.rate, self.latency, self.no_wait = rate_GBs, latency_us, no_wait
        self.log = []    # (nbytes, modeled us) per collective

    def issue(self, nbytes: int, deliver, tensors=(), async_op: bool = True):
        cur = torch.cuda.current_stream(self.device)
        ready = torch.cuda.Event()
        ready.record(cur)
        us = _wire_us(nbytes, self.rate, self.latency)
        self.log.append((nbytes, us))
        with torch.cuda.stream(self.side):
            self.side.wait_event(ready)
            spin_us(us, self.device)
            deliver()
            for t in tensors:
                if t is not None and t.is_cuda:
                    t.record_stream(self.side)
            done = torch.cuda.Event()
            done.record(self.side)
        w = (NoWaitWork if self.no_wait else Work)([done])
        if not async_op:
            Work([done]).wait()
            return None
        return w


class ThreadFabric:
    """The collectives of `distributed.py` (all_to_all_single, all_gather_into_tensor,
    all-reduce MAX) between `world` ranks that run as threads of this process on
    one GPU.  Each rank thread calls ``bind(rank)`` first; it then runs on its own
    current stream, and every collective it issues is delivered on its own side
    stream after every participant's queued work (their ready events) and a
    modeled wire spin.  A rank's wait() waits for every rank's delivery of that
    collective, since they all read its input."""

    def __init__(self, world: int, device, rate_GBs: float | None = None,
                 latency_us: float = 10.0, fixed_us: float | None = None, no_wait: bool = False,
                 sync: bool = False, timeout_s: float = 120.0):
        """rate_GBs / latency_us: the modeled per-rank wire (bytes a rank receives
        / rate + latency); fixed_us: a fixed spin per collective instead; sync:
        gloo's semantics (every collective waited before the call returns);
        no_wait: handles whose wait() does nothing (negative control)."""
        self.world, self.device = world, torch.device(device)
        self.sync = sync
        # torch caches the device count only once initialised, and a first count
        # taken on a worker thread came back 0 on the GPU box ("Invalid device id"
        # from get_device_properties): take it here, on the calling thread
        torch.cuda.init()
        torch.cuda.get_device_properties(self.device)
        self.rate, self.latency, self.fixed_us, self.no_wait = rate_GBs, latency_us, fixed_us, no_wait
        self._bar = threading.Barrier(world, timeout=timeout_s)
        self._slots = [None] * world
        self._done = [None] * world
        self._tl = threading.local()
        self.streams = [torch.cuda.Stream(self.device) for _ in range(world)]
        self.sides = [torch.cuda.Stream(self.device) for _ in range(world)]
        self.calls = [0] * world
        self.waited = []     # every async handle issued (checked by the tests)

    # ------------------------------------------------------------- plumbing
    def streams_concurrent(self, spin_ms: float = 20.0) -> bool:
        """Whether every rank's compute stream really runs beside its side stream:
        HIP maps streams onto a few hardware queues (GPU_MAX_HW_QUEUES), and two
        streams on one queue run in order -- correct, but not concurrent.  A long
        spin on the side stream and a tiny op on the compute stream: concurrent when
        the tiny op completes well before the spin."""
        import time
        ok = True
        for r in range(self.world):
            with torch.cuda.stream(self.sides[r]):
                spin_us(spin_ms * 1e3, self.device)
            done = torch.cuda.Event()
            with torch.cuda.stream(self.streams[r]):
                torch.cuda._sleep(1)
                done.record()
            t0 = time.perf_counter()
            done.synchronize()
            ok = ok and (time.perf_counter() - t0) * 1e3 < spin_ms / 2
            torch.cuda.synchronize(self.device)
        return ok

    def bind(self, rank: int):
        self._tl.rank = rank
        torch.cuda.set_stream(self.streams[rank])

    @property
    def rank(self) -> int:
        return self._tl.rank

    def _us(self, nbytes):
        if self.fixed_us is not None:
            return self.fixed_us
        return _wire_us(nbytes, self.rate, self.latency)

    def _exchange(self, payload, deliver, out, inp, nbytes, async_op):
        """Barrier-synchronised collective: every rank posts (payload, ready
        event); each then delivers its own output on its side stream."""
        r = self.rank
        cur = torch.cuda.current_stream(self.device)
        ready = torch.cuda.Event()
        ready.record(cur)
        self._slots[r] = (payload, ready)
        self._bar.wait()
        slots = list(self._slots)
        side = self.sides[r]
        with torch.cuda.stream(side):
            for _, ev in slots:
                side.wait_event(ev)
            spin_us(self._us(nbytes), self.device)
            deliver(slots)
            for t in (out, inp):
                if t is not None and t.is_cuda:
                    t.record_stream(side)
            for p, _ in slots:              # the peers' inputs are read here too
                t = p[0] if isinstance(p, tuple) else p
                if isinstance(t, torch.Tensor) and t.is_cuda:
                    t.record_stream(side)
            done = torch.cuda.Event()
            done.record(side)
        self._done[r] = done
        self._bar.wait()
        events = list(self._done)
        self._bar.wait()                    # nobody overwrites the slots before all read them
        self.calls[r] += 1
        if not async_op or self.sync:
            Work(events).wait()
            if async_op:
                w = Work([])
                w.waited = True
                return w
            return out
        w = (NoWaitWork if self.no_wait else Work)(events)
        self.waited.append(w)
        return w

    # ----------------------------------------------------------- collectives
    def a2a(self, out, inp, out_split=None, in_split=None, async_op=False):
        """all_to_all_single(out, inp, out_split, in_split)."""
        world, r = self.world, self.rank
        n_in, n_out = inp.shape[0], out.shape[0]
        in_split = list(in_split) if in_split is not None else [n_in // world] * world
        out_split = list(out_split) if out_split is not None else [n_out // world] * world
        row = out[0].numel() * out.element_size() if n_out else 0

        def deliver(slots):
            o = 0
            for q in range(world):
                q_inp, q_split = slots[q][0]
                s = sum(q_split[:r])
                n = q_split[r]
                if n != out_split[q]:
                    raise RuntimeError(f"rank {r}: peer {q} sends {n} rows, expected {out_split[q]}")
                if n:
                    out[o:o + n].copy_(q_inp[s:s + n])
                o += n

        nbytes = (sum(out_split) - out_split[r]) * row
        return self._exchange((inp, in_split), deliver, out, inp, nbytes, async_op)

    def ag(self, out, inp, async_op=False):
        """all_gather_into_tensor(out, inp): rank q's chunk at rows q * n."""
        n = inp.shape[0]

        def deliver(slots):
            for q in range(self.world):
                out[q * n:(q + 1) * n].copy_(slots[q][0][0])

        nbytes = (self.world - 1) * inp.numel() * inp.element_size()
        return self._exchange((inp, None), deliver, out, inp, nbytes, async_op)

    def max_over_ranks(self, *xs: float):
        """The all-reduce MAX of PartitionedMaxK._max_over_ranks (host values)."""
        r = self.rank
        self._slots[r] = (list(xs), None)
        self._bar.wait()
        vals = [max(self._slots[q][0][i] for q in range(self.world)) for i in range(len(xs))]
        self._bar.wait()
        return vals[0] if len(xs) == 1 else vals

    def run(self, fn):
        """Run fn(rank) on `world` threads (each bound to its rank and streams);
        returns the list of results, re-raising the first exception."""
        res, err = [None] * self.world, [None] * self.world

        def body(q):
            try:
                self.bind(q)
                res[q] = fn(q)
                torch.cuda.current_stream(self.device).synchronize()
            except BaseException as e:   # noqa: BLE001 -- re-raised below
                err[q] = e
                self._bar.abort()

        th = [threading.Thread(target=body, args=(q,)) for q in range(self.world)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for e in err:
            if e is not None and not isinstance(e, threading.BrokenBarrierError):
                raise e
        for e in err:
            if e is not None:
                raise e
        return res


def install(fabric, D):
    """Route distributed.py's collectives (module `D`) through `fabric`;
    returns a function that restores the originals."""
    saved = (D.a2a, D.ag, D.PartitionedMaxK._max_over_ranks)
    D.a2a = fabric.a2a
    D.ag = fabric.ag
    D.PartitionedMaxK._max_over_ranks = lambda self, *xs: (
        (xs[0] if len(xs) == 1 else list(xs)) if self.world == 1 else fabric.max_over_ranks(*xs))

    def restore():
        D.a2a, D.ag, D.PartitionedMaxK._max_over_ranks = saved
    return restore
