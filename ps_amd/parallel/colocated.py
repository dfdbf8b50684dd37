"""Co-located parameter server over collectives -- the MI355X hot path.

Reference architecture (structure.png): W worker processes push per-key
gradients to S server processes over gRPC, the servers apply the optimizer, workers pull
the weights back and meet at a barrier (store/KVStore.java:240-268, net/PServer.java:164-283).

MI355X-native design: every GPU process is a worker AND the server of a range partition
(registry.py).  Per bucket, in the order buckets become ready during backward:

    push  = reduce-scatter of the bf16 gradient bucket       (RCCL over xGMI, comm stream)
    serve = fused HIP optimizer on the owned fp32 master chunk; it writes the updated
            weights straight into the owned chunk of the bf16 pull buffer   (same stream)
    pull  = all-gather of the bucket from every owner         (RCCL, same stream)

all overlapped with the rest of backward: the comm stream waits on an event recorded on the
compute stream when the bucket's last gradient has been accumulated
(``register_post_accumulate_grad_hook``), and the compute stream waits on the round's
completion event only before the forward that needs the new weights.

Consistency (SURVEY §2.3, quirks Q1-Q3 fixed):
  * BSP  (staleness=0): forward t+1 sees exactly the weights after every push of step t.
  * SSP  (staleness=s): forward t+1 uses weights version max(0, t+1-s); rounds stay in
    flight for up to s steps.  Weight and gradient buffers are rings of s+1 slots so the
    in-flight pull never writes the buffer the compute stream is reading.  A worker that
    runs ahead blocks on the completion event of round t-s, i.e. when its clock leads the
    slowest worker by more than s -- the SSP bound, enforced by the collective itself.
  * Gradient accumulators are zeroed every round and averaged over exactly W workers.

Gradient landing (no per-parameter accumulate kernels): ``p.grad`` is None when backward
starts, so autograd's AccumulateGrad adopts each freshly computed gradient without a kernel;
the post-accumulate hook parks it, and when a bucket's last key is ready ONE multi-tensor copy
(``torch._foreach_copy_``) lands all of them in the flat bucket, after which ``p.grad`` is the
bucket view.  4-D conv weights with spatial extent (3x3) are stored channels_last inside the
flat buffers, so the replica the forward reads and the gradient MIOpen returns already have
the layout the convolution wants -- no per-step weight / gradient transposes.  Keys that got
no gradient in a step are zero-filled at launch.

Options: global-norm clipping (two-phase: push all, norm, then serve+pull), 1-bit
compressed push with error feedback (compress="onebit": bits all-to-all to the owners +
owner-side unpack-reduce kernel; ``compress_warmup`` full-precision rounds first),
arbitrary per-key-prefix updaters (resolve_updater).
"""
from __future__ import annotations

import contextlib
import os

import time
from collections import deque
from functools import partial
from typing import Dict, List, Optional, Union

import torch

from ..obs import trace as _trace
from ..ops import compress as _cmp
from ..ops import reduce as _red
from ..ops import side_stream as _side
from .registry import Registry
from .transport import Transport
from .updaters import Updater, resolve_updater


class ColocatedPS:
    def __init__(self, model: torch.nn.Module, updaters: Union[Updater, Dict[str, Updater]],
                 transport: Optional[Transport] = None, *, bucket_mb: float = 32.0, last_bucket_mb: float = 4.0,
                 staleness: int = 0, clip_norm: Optional[float] = None, compress: Optional[str] = None,
                 average: bool = True, broadcast_init: bool = True, overlap: bool = True, timing: bool = False,
                 compress_warmup: int = 0, split_comm: Optional[bool] = None, plane: Optional[str] = None,
                 timeout_s: float = 600.0, reduce_fp32: Optional[bool] = None,
                 ef_dtype: Optional[torch.dtype] = None, onebit_momentum: Optional[float] = None):
        self.model = model
        self.t = transport or Transport()
        self.world, self.rank = self.t.world, self.t.rank
        self.updaters = updaters if isinstance(updaters, dict) else {"default": updaters}
        self.staleness = int(staleness)
        if self.staleness < 0:
            raise ValueError("staleness must be >= 0")
        self.nslots = self.staleness + 1
        self.clip_norm = clip_norm
        self.compress = compress
        if compress not in (None, "onebit"):
            raise ValueError(f"unknown compression {compress!r}")
        # full-precision rounds before the 1-bit push takes over: the
        # error-feedback state starts from zero at the switch
        self.compress_warmup = int(compress_warmup)
        # 1-bit Adam (updaters.OneBitAdamUpdater): every worker keeps its momentum
        # m = beta1 m + (1 - beta1) g from round 0 and, after the warm-up, pushes the error-compensated
        # 1-bit MOMENTUM; the owners' Adam runs with beta1 = 0 and a frozen variance from then on
        self.onebit_momentum = None if onebit_momentum is None else float(onebit_momentum)
        if self.onebit_momentum is not None:
            from .updaters import OneBitAdamUpdater

            if compress != "onebit":
                raise ValueError("onebit_momentum needs compress='onebit'")
            bad = [k for k, u in self.updaters.items()
                   if not isinstance(u, OneBitAdamUpdater) or u.warmup != self.compress_warmup
                   or u.beta1 != self.onebit_momentum]
            if bad or len({u.refresh for u in self.updaters.values()}) != 1:
                raise ValueError(f"onebit_momentum: every updater must be OneBitAdamUpdater(warmup=compress_warmup="
                                 f"{self.compress_warmup}, beta1={self.onebit_momentum}), one refresh; not {bad}")
            self._full_round = next(iter(self.updaters.values())).full_round
        self.average = average
        self.overlap = overlap
        # collective plane: reduce-scatter bf16 buckets in fp32 when reduce_fp32 (the W-way sum is
        # otherwise rounded in bf16 by RCCL); the xGMI plane always sums in fp32 on the owner
        self.reduce_fp32 = bool(reduce_fp32)
        self.accumulating = False  # micro-batch accumulation: hooks stay quiet until the last one
        params = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        if not params:
            raise ValueError("model has no trainable parameters")
        self.device = params[0][1].device
        self.gpu = self.device.type == "cuda"
        align = 1024 if compress == "onebit" else 64
        self.reg = Registry(self.world, int(bucket_mb * 2**20), align, int(last_bucket_mb * 2**20) or None)
        for n, p in reversed(params):
            self.reg.add(n, p.shape, p.dtype)
        self.reg.finalize()
        self.params = dict(params)
        # keys stored channels_last in the flat buffers (element order O, kh, kw, I)
        self.cl_keys = {n for n, p in params if _wants_channels_last(p)}
        R = self.reg
        # ---------------- data plane: one-sided xGMI plane (plane.py) or collectives (transport)
        from .plane import XgmiPlane, env_plane, plane_available

        req = plane or env_plane()
        if req not in ("auto", "xgmi", "collective"):
            raise ValueError(f"unknown plane {req!r}")
        use_plane = self.world > 1 and (req == "xgmi" or (req == "auto" and self.gpu
                                                             and plane_available(self.t, self.device)))
        self.plane = None
        if use_plane:
            from .plane import PlaneUnavailable

            try:
                self.plane = XgmiPlane(self.t, R, self.device, self.nslots, onebit=compress == "onebit",
                                       clip_norm=clip_norm, average=average, timeout_s=timeout_s)
            except PlaneUnavailable as e:  # raised on every rank alike: the fallback is uniform
                if req == "xgmi":
                    raise
                import sys

                print(f"[ps_amd] {e}; using the collective data plane", file=sys.stderr, flush=True)
        self.plane_kind = "xgmi" if self.plane is not None else ("collective" if self.world > 1 else "local")
        # ---------------- replica buffers (rings of s+1 slots)
        if self.plane is not None:
            self.wbuf = self.plane.slots("w")
            self.gbuf = self.plane.slots("g")
        else:
            self.wbuf = {g: [torch.zeros(R.group_size[g], dtype=R.group_dtype[g], device=self.device)
                             for _ in range(self.nslots)] for g in R.group_size}
            self.gbuf = {g: [torch.zeros(R.group_size[g], dtype=R.group_dtype[g], device=self.device)
                             for _ in range(self.nslots)] for g in R.group_size}
        with torch.no_grad():
            for n, p in params:
                ki = R.keys[n]
                src = p.detach().permute(0, 2, 3, 1) if n in self.cl_keys else p.detach()
                self.wbuf[ki.group][0][ki.offset:ki.offset + ki.numel].view(src.shape).copy_(src)
            if broadcast_init and self.plane is not None:
                self.plane.broadcast_weights(self.wbuf, src=0)
            elif broadcast_init:
                for g in self.wbuf:
                    self.t.broadcast(self.wbuf[g][0], src=0)
            for g in self.wbuf:
                for s in range(1, self.nslots):
                    self.wbuf[g][s].copy_(self.wbuf[g][0])
        # ---------------- server state: fp32 master + optimizer state for the owned chunks
        self.master: List[torch.Tensor] = []
        self.segs: List[List[tuple]] = []  # per bucket: [(updater, lo, hi)] chunk-local
        self.states: List[List[List[torch.Tensor]]] = []
        self.gshard: List[Optional[torch.Tensor]] = []
        for b in R.buckets:
            lo, hi = b.owner_range(self.rank)
            m = self.wbuf[b.group][0][lo:hi].float().clone()
            self.master.append(m)
            segs = []
            for k, a, z in R.segments(b.index, self.rank):
                u = resolve_updater(k, self.updaters)
                la, lz = a - lo, z - lo
                if segs and segs[-1][0] is u and segs[-1][2] == la:
                    segs[-1] = (u, segs[-1][1], lz)
                else:
                    segs.append((u, la, lz))
            if not segs:  # chunk is pure padding: give it to the default updater
                segs = [(resolve_updater(b.keys[0], self.updaters), 0, hi - lo)]
            # extend first/last segment over leading/trailing padding
            segs[0] = (segs[0][0], 0, segs[0][2])
            segs[-1] = (segs[-1][0], segs[-1][1], hi - lo)
            self.segs.append(segs)
            self.states.append([u.new_states(m[a:z]) for (u, a, z) in segs])
            if self.world > 1 and self.plane is None:
                gdt = torch.float32 if (self.reduce_fp32 and compress is None) else R.group_dtype[b.group]
                self.gshard.append(torch.empty(b.chunk, dtype=gdt, device=self.device))
            else:
                self.gshard.append(None)
        # 1-bit compression state: error-feedback buffer per bucket (full bucket; fp32, or bf16 via
        # ``ef_dtype`` -- Llama-3-8B: 16 instead of 32 GB per rank); with the plane the packed words
        # / scales live in its arena (one per gradient slot)
        self.ef_dtype = ef_dtype or torch.float32
        if self.ef_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"error-feedback dtype {ef_dtype} (fp32 or bf16)")
        # the plane path packs on its own stream behind each bucket's landing event, so the
        # 1-bit pack + error feedback never sits in the backward's stream
        self.pack_stream = None
        # worker momenta of 1-bit Adam, in the error-feedback dtype (the pack kernel reads both alike)
        self.wmom = ([torch.zeros(b.size, dtype=self.ef_dtype, device=self.device) for b in R.buckets]
                     if self.onebit_momentum is not None else None)
        if compress == "onebit" and self.plane is not None:
            self.err = [torch.zeros(b.size, dtype=self.ef_dtype, device=self.device) for b in R.buckets]
            if self.gpu:
                self.pack_stream = torch.cuda.Stream(device=self.device)
        elif compress == "onebit":
            self.err = [torch.zeros(b.size, dtype=self.ef_dtype, device=self.device) for b in R.buckets]
            self.cwords = []
            self.cscales = []
            for b in R.buckets:
                nw, ns = _cmp.packed_sizes(b.size)
                self.cwords.append((torch.empty(nw, dtype=torch.int64, device=self.device),
                                    torch.empty(nw, dtype=torch.int64, device=self.device)))
                self.cscales.append((torch.empty(ns, dtype=torch.float32, device=self.device),
                                     torch.empty(ns, dtype=torch.float32, device=self.device)))
        # ---------------- clipping scratch
        if clip_norm is not None:
            self._sq = torch.zeros(1, dtype=torch.float32, device=self.device)
            self._factor = torch.ones(1, dtype=torch.float32, device=self.device)
        # ---------------- step state
        self.round = 0  # PS clock: number of completed pushes
        self.wslot = 0
        self.gslot = 0
        self.pending = [len(b.keys) for b in R.buckets]
        self.launched = [False] * len(R.buckets)
        self._key_bucket = {n: R.keys[n].bucket for n in self.params}
        self._landing: List[Dict[str, torch.Tensor]] = [dict() for _ in R.buckets]  # parked grads
        self.comm = torch.cuda.Stream(device=self.device) if self.gpu else None
        # separate push / pull communicators: the all-gather of bucket b runs on
        # its own communicator + stream, so the reduce-scatter of bucket b+1 need not wait behind
        # it; opt-in (split_comm=True) -- the default single communicator is what the measured
        # multi-GPU configs use
        self.split_comm = bool(split_comm) and self.world > 1
        self.tpull = self.t.split() if self.split_comm else self.t
        self.comm_pull = torch.cuda.Stream(device=self.device) if (self.gpu and self.split_comm) else self.comm
        # one worker: nothing crosses a wire, so each bucket's serve runs inline on the stream that
        # landed it (compute, or the side stream for weight gradients).  A separate comm stream
        # only adds cross-queue event waits at the step boundary: the last serve and the next
        # forward each waited 0.1-0.6 ms for an event already signalled on another queue
        # (ResNet-50 bs1024, profiles/r6_step_boundary_gap.txt)
        # Large models keep the comm stream: their serve (Llama-3-8B: ~50-130 ms of AdamW over 8B
        # masters) is worth overlapping with backward (profiles/r4_llama_serve_overlap.txt).
        self.inline_serve = (self.gpu and self.world == 1 and self.plane is None and clip_norm is None
                             and sum(b.size for b in R.buckets) <= (1 << 28))
        # per parameter group, the bucket that holds its first layers (backward order: it fires last)
        last = {}
        for i, bk in enumerate(R.buckets):
            if bk.group not in last or bk.start > R.buckets[last[bk.group]].start:
                last[bk.group] = i
        self._group_last = set(last.values())
        self.round_events: deque = deque()
        # host run-ahead bound (GPU), PS_AMD_MAX_INFLIGHT (0 = unbounded): finish_step waits on the
        # host until the step max_inflight - 1 steps back is done.  The host issues a ResNet-50
        # step in ~10 ms against a 62 ms GPU step (bs1024), so unbounded it runs many steps ahead;
        # then, once per process at a random point in the first ~30 steps, the runtime stalls for
        # 2-4 s (2 of 3 runs with --warmup 5 timed 6.2-6.9K img/s instead of 16.5K; with the
        # bound at 2: 3 of 3 normal, and no steady-state cost -- profiles/r5_run_ahead_ab.txt).
        self.max_inflight = int(os.environ.get("PS_AMD_MAX_INFLIGHT", "2"))
        self._host_events: deque = deque()
        self.stats = {"exposed_wait_ms": 0.0, "rounds": 0}
        # fault injection (PS_AMD_FAULT / HIPPS_FAULT): kill at a step, delay pushes
        from ..utils.fault import FaultInjector

        fi = FaultInjector(rank=self.rank)
        self.fault = fi if fi.spec else None
        # per-step phase timing: device events on the comm stream around push /
        # serve / pull of every bucket, plus backward-end vs round-end for the exposed tail
        self.timing = timing or os.environ.get("PS_AMD_TIMING", "0") == "1"
        self._marks: List[tuple] = []  # (name, event or perf_counter) of the current step
        self._tsum: Dict[str, float] = {}
        self._tsteps = 0
        self._prev_marks: List[tuple] = []
        self._bind(self.wslot, self.gslot)
        self._mark("step0")
        if self.plane is not None:
            self.plane.attach(self)
        self._hooks = [p.register_post_accumulate_grad_hook(partial(self._on_ready, n)) for n, p in params]

    # ------------------------------------------------------------------ views
    def _view(self, buf: Dict[str, List[torch.Tensor]], slot: int, name: str) -> torch.Tensor:
        ki = self.reg.keys[name]
        flat = buf[ki.group][slot][ki.offset:ki.offset + ki.numel]
        if name in self.cl_keys:
            o, i, kh, kw = ki.shape
            return flat.view(o, kh, kw, i).permute(0, 3, 1, 2)
        return flat.view(ki.shape)

    def _bind(self, wslot: int, gslot: int) -> None:
        from ..ops.linear import GradDst

        for n, p in self.params.items():
            p.data = self._view(self.wbuf, wslot, n)
            p.grad = None  # AccumulateGrad adopts the fresh gradient; _land() copies it in
            if self.gpu and n not in self.cl_keys:
                # where this step's gradient lives: a producer that knows it (ops/linear.py
                # PsLinear) writes there directly and _land() has nothing to copy
                ki = self.reg.keys[n]
                d = getattr(p, "_ps_gdst", None)
                if d is None:
                    p._ps_gdst = GradDst(self.gbuf[ki.group][gslot], ki.offset, ki.numel, ki.shape)
                else:
                    d.buf, d.off, d.claimed = self.gbuf[ki.group][gslot], ki.offset, False

    def weight(self, name: str) -> torch.Tensor:
        """Current replica weights of key ``name`` (the pulled version)."""
        return self._view(self.wbuf, self.wslot, name)

    # ------------------------------------------------------------------ push path
    def push_key(self, name: str, grad: torch.Tensor) -> None:
        """Key-level push (parallel/gpu_kvstore.py): park ``grad`` for key ``name`` as the
        backward hook does; the key's bucket leaves once its last key arrived.  A second push of
        a key in the same round adds to the parked gradient while its bucket has not left."""
        p = self.params[name]
        b = self._key_bucket[name]
        g = grad.detach().to(device=p.device, dtype=p.dtype).reshape(p.shape)
        if name in self._landing[b]:
            self._landing[b][name] = self._landing[b][name] + g
            return
        if self.launched[b]:
            raise RuntimeError(f"key {name!r} was already pushed this round (its bucket has left)")
        p.grad = g
        self._on_ready(name, p)

    def _on_ready(self, name: str, p: torch.Tensor) -> None:
        if self.accumulating:
            return
        b = self._key_bucket[name]
        if name not in self._landing[b]:
            self.pending[b] -= 1
        self._landing[b][name] = p.grad
        if self.pending[b] == 0 and self.overlap:
            self._launch(b)

    def _land(self, b: int) -> None:
        """Copy the bucket's parked gradients into its gradient slot (one multi-tensor kernel on
        the compute stream) and rebind ``p.grad`` to the bucket views; zero keys without one."""
        parked = self._landing[b]
        dst, src = [], []
        for n in self.reg.buckets[b].keys:
            v = self._view(self.gbuf, self.gslot, n)
            g = parked.get(n)
            if g is None:
                v.zero_()
            elif g.data_ptr() != v.data_ptr():
                dst.append(v)
                src.append(g)
            self.params[n].grad = v
        if dst:
            torch._foreach_copy_(dst, src)
        self._landing[b] = {}

    def _launch(self, b: int, in_backward: bool = True) -> None:
        if self.launched[b]:
            return
        self.launched[b] = True
        # after backward (finish_step) the compute stream has already joined the side stream
        # (ops/side_stream.py end-of-backward callback): a bucket launched then lands on the compute
        # stream directly -- routing it through the side stream cost two cross-queue event waits
        # at the step boundary (0.56 + 0.12 ms per ResNet-50 step, profiles/r6_step_boundary_gap.txt)
        side = _side.active(self.device) if (self.gpu and in_backward) else None
        if side is not None and not any(_side.produced_on_side(g) for g in self._landing[b].values()):
            side = None  # every gradient of the bucket came from the compute stream
        if side is not None and b in self._group_last:
            # the last bucket of its group holds the first layers: its gradients complete the
            # backward, so the compute stream has nothing left to overlap -- it joins the side stream
            # (whose weight gradients are done by now) and serves the bucket itself; the side stream
            # serving it left the next forward waiting ~0.1 ms on a cross-queue event
            torch.cuda.current_stream(self.device).wait_stream(side)
            side = None
        if side is not None:
            # some of the bucket's gradients are weight gradients still in flight on the side
            # stream (ops/side_stream.py): land and push from that stream, after the compute
            # stream's part of the bucket, so the data-gradient chain never waits for them
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            side.wait_event(ev)
            for g in self._landing[b].values():
                if g is not None:
                    g.record_stream(side)
            with torch.cuda.stream(side):
                self._launch_body(b)
        else:
            self._launch_body(b)

    def _launch_body(self, b: int) -> None:
        self._land(b)
        if self.fault is not None:
            self.fault.before_push()
        if self.plane is not None:
            onebit = self._onebit_round()
            if onebit or self.wmom is not None:
                bk = self.reg.buckets[b]
                gin = self.gbuf[bk.group][self.gslot][bk.start:bk.start + bk.size]
                if self.pack_stream is not None:  # behind the landing, off the backward's stream
                    ev = torch.cuda.Event()
                    ev.record(torch.cuda.current_stream(self.device))
                    self.pack_stream.wait_event(ev)
                with (torch.cuda.stream(self.pack_stream) if self.pack_stream is not None
                      else contextlib.nullcontext()):
                    self._mark("pack0")
                    if onebit:  # sign bits + scales + error feedback (of the momentum, 1-bit Adam)
                        words, scales = self.plane.words(b, self.gslot)
                        _cmp.onebit_pack(gin, self.err[b], words, scales,
                                         None if self.wmom is None else self.wmom[b], self.onebit_momentum or 0.0)
                    else:  # 1-bit Adam warm-up: the momentum only, the push is the full gradient
                        _cmp.onebit_momentum(gin, self.wmom[b], self.onebit_momentum)
                    self._mark("pack1")
                    with _trace.range(f"ps.push.b{b}"):  # the push's landing event: after the pack
                        self.plane.push(b, self.round, self.gslot, (self.round + 1) % self.nslots, onebit)
                return
            with _trace.range(f"ps.push.b{b}"):
                self.plane.push(b, self.round, self.gslot, (self.round + 1) % self.nslots, onebit)
            return
        if self.gpu and self.inline_serve:
            with _trace.range(f"ps.serve_pull.b{b}"):
                self._serve_pull(b)
            return
        if self.gpu:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self.comm.wait_event(ev)
            with torch.cuda.stream(self.comm), _trace.range(f"ps.push.b{b}"):  # roctx
                self._mark("push0")
                self._push(b)
                self._mark("push1")
            if self.clip_norm is None:
                if self.comm_pull is not self.comm:
                    pev = torch.cuda.Event()
                    pev.record(self.comm)
                    self.comm_pull.wait_event(pev)
                with torch.cuda.stream(self.comm_pull), _trace.range(f"ps.serve_pull.b{b}"):
                    self._serve_pull(b)
        else:
            self._mark("push0")
            self._push(b)
            self._mark("push1")
            if self.clip_norm is None:
                self._serve_pull(b)

    # ------------------------------------------------------------------ timing
    def _mark(self, name: str) -> None:
        if not self.timing:
            return
        if self.gpu:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()  # current stream (comm inside _launch, compute in finish_step)
            self._marks.append((name, ev))
        else:
            self._marks.append((name, time.perf_counter()))

    def _close_timing(self) -> None:
        """Fold the finished step's marks into the running sums (synchronizes on them)."""
        if not self._marks:
            return
        def ms(a, b):
            return a.elapsed_time(b) if self.gpu else (b - a) * 1e3
        if self.gpu:
            self._marks[-1][1].synchronize()
        # only the phases that were marked: the xGMI plane path returns before any push / serve /
        # pull mark (its phases are the plane's own device-timed statistics, ``plane_stats``), so
        # its record carries no placeholder zeros for them
        acc: Dict[str, float] = {}
        last = {}
        for name, t in self._marks:
            if name == "push1":
                acc["push_ms"] = acc.get("push_ms", 0.0) + ms(last["push0"], t)
            elif name == "serve1":
                acc["serve_ms"] = acc.get("serve_ms", 0.0) + ms(last.get("push1", last.get("serve0")), t)
            elif name == "pull1":
                acc["pull_ms"] = acc.get("pull_ms", 0.0) + ms(last["serve1"], t)
            elif name == "pack1":  # 1-bit pack + error feedback of one bucket (plane path)
                acc["pack_ms"] = acc.get("pack_ms", 0.0) + ms(last["pack0"], t)
                acc["packs"] = acc.get("packs", 0.0) + 1.0
            last[name] = t
        if "bwd_end" in last and "round_end" in last:
            acc["exposed_comm_ms"] = max(0.0, ms(last["bwd_end"], last["round_end"]))
        if "step0" in last and "bwd_end" in last:
            acc["fwd_bwd_ms"] = ms(last["step0"], last["bwd_end"])
        for k, v in acc.items():
            self._tsum[k] = self._tsum.get(k, 0.0) + v
        self._tsteps += 1
        self._marks = []

    def timing_summary(self, reset: bool = True) -> Dict[str, float]:
        """Mean per-step phase times (ms) since the last reset: fwd_bwd, push (reduce-scatter),
        serve (owner optimizer), pull (all-gather) summed over buckets, and the exposed tail of
        the round after backward.  Enable with ``timing=True`` or PS_AMD_TIMING=1."""
        if self._prev_marks:  # the last completed step (the current one is still open)
            cur, self._marks = self._marks, self._prev_marks
            self._close_timing()
            self._marks, self._prev_marks = cur, []
        out = {k: v / max(1, self._tsteps) for k, v in self._tsum.items()}
        if reset:
            self._tsum, self._tsteps = {}, 0
        return out

    def _push(self, b: int) -> None:
        bk = self.reg.buckets[b]
        gin = self.gbuf[bk.group][self.gslot][bk.start:bk.start + bk.size]
        if self.world == 1:
            if self.wmom is not None:  # 1-bit Adam with nothing to push: the owner still gets the momentum
                _cmp.onebit_momentum(gin, self.wmom[b], self.onebit_momentum)
                if self._onebit_round(any_world=True):
                    gin.copy_(self.wmom[b])
            return
        if self._onebit_round():
            self._push_onebit(b, gin)
            return
        if self.wmom is not None:  # 1-bit Adam warm-up: keep the worker momentum, push the gradient
            _cmp.onebit_momentum(gin, self.wmom[b], self.onebit_momentum)
        if self.gshard[b].dtype != gin.dtype:  # fp32 reduction of a bf16 bucket
            self.t.reduce_scatter(self.gshard[b], gin.float())
        else:
            self.t.reduce_scatter(self.gshard[b], gin)

    def _onebit_round(self, any_world: bool = False) -> bool:
        """This round's push is 1-bit: past the warm-up, and (1-bit Adam) not a variance-refresh round."""
        if self.compress != "onebit" and not (any_world and self.wmom is not None):
            return False
        if self.wmom is not None:
            return not self._full_round(self.round + 1)
        return self.round >= self.compress_warmup

    def _push_onebit(self, b: int, gin: torch.Tensor) -> None:
        """Compressed push: sign bits + chunk scales, all-to-all to the owners, owner decodes
        and sums the W contributions in fixed rank order."""
        bk = self.reg.buckets[b]
        words, rwords = self.cwords[b]
        scales, rscales = self.cscales[b]
        _cmp.onebit_pack(gin, self.err[b], words, scales, None if self.wmom is None else self.wmom[b],
                         self.onebit_momentum or 0.0)
        self.t.all_to_all(rwords, words)
        self.t.all_to_all(rscales, scales)
        nw_chunk = bk.chunk // 64
        ns_chunk = bk.chunk // _cmp.CHUNK
        _cmp.onebit_unpack_reduce(rwords.view(self.world, nw_chunk), rscales.view(self.world, ns_chunk),
                                  self.gshard[b], 1.0, False)

    def _grad_shard(self, b: int) -> torch.Tensor:
        if self.world == 1:
            bk = self.reg.buckets[b]
            return self.gbuf[bk.group][self.gslot][bk.start:bk.start + bk.size]
        return self.gshard[b]

    def _serve_pull(self, b: int) -> None:
        bk = self.reg.buckets[b]
        lo, hi = bk.owner_range(self.rank)
        nxt = (self.round + 1) % self.nslots
        wfull = self.wbuf[bk.group][nxt]
        own = wfull[lo:hi]
        g = self._grad_shard(b)
        gscale = 1.0 / self.world if self.average else 1.0
        gst = self._factor if self.clip_norm is not None else None
        self._mark("serve0")
        for (u, a, z), st in zip(self.segs[b], self.states[b]):
            u.step_flat(self.master[b][a:z], st, g[a:z], wout=own[a:z], gscale=gscale, gscale_t=gst,
                        step=self.round + 1)
        self._mark("serve1")
        self.tpull.all_gather(wfull[bk.start:bk.start + bk.size], own)
        self._mark("pull1")

    def _clip_and_serve(self) -> None:
        self._sq.zero_()
        for b in range(len(self.reg.buckets)):
            _red.sumsq(self._grad_shard(b), self._sq, accumulate=True)
        self.t.all_reduce(self._sq)
        # norm of the averaged gradient = norm(sum) / W
        scale = self.world if self.average else 1
        _red.clip_factor(self._sq, float(self.clip_norm) * scale, self._factor)
        for b in range(len(self.reg.buckets)):
            self._serve_pull(b)

    # ------------------------------------------------------------------ step boundary
    def finish_step(self) -> None:
        """End of a worker step: flush buckets that did not fire, run the round's remaining
        phases, advance the PS clock and bind the weights the next forward may use."""
        if self.fault is not None:
            self.fault.at_step(self.round)
        _trace.mark(f"ps.finish_step.r{self.round}")
        if self.timing:
            self._mark("bwd_end")
        for b in range(len(self.reg.buckets)):
            if not self.launched[b]:
                self._launch(b, in_backward=False)
        if self.plane is not None:
            self._finish_plane_round()
            return
        if self.clip_norm is not None:
            if self.gpu:
                self.comm_pull.wait_stream(self.comm)
                with torch.cuda.stream(self.comm_pull):
                    self._clip_and_serve()
            else:
                self._clip_and_serve()
        if self.gpu:
            if self.comm_pull is not self.comm:
                self.comm_pull.wait_stream(self.comm)  # the round ends when both streams are done
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device) if self.inline_serve else self.comm_pull)
            self.round_events.append(ev)
        if self.timing:
            if self.gpu:
                with torch.cuda.stream(torch.cuda.current_stream(self.device) if self.inline_serve else self.comm_pull):
                    self._mark("round_end")
            else:
                self._mark("round_end")
        r = self.round
        self.round += 1
        self.stats["rounds"] += 1
        # weights version for the next forward
        v = max(0, self.round - self.staleness)
        need_round = v - 1  # round that produced version v
        if self.gpu:
            while self.round_events and (r - len(self.round_events) + 1) <= need_round:
                ev = self.round_events.popleft()
                torch.cuda.current_stream(self.device).wait_event(ev)
        self.wslot = v % self.nslots
        self.gslot = self.round % self.nslots
        # no zero-fill of the next gradient slot: _land() overwrites every key region (padding is
        # never written and stays zero)
        self.pending = [len(b.keys) for b in self.reg.buckets]
        self.launched = [False] * len(self.reg.buckets)
        self._bind(self.wslot, self.gslot)
        self._bound_run_ahead()
        if self.timing:
            self._close_timing_deferred()

    def _bound_run_ahead(self) -> None:
        if not self.gpu or self.max_inflight <= 0 or torch.cuda.is_current_stream_capturing():
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._host_events.append(ev)
        while len(self._host_events) >= self.max_inflight:
            self._host_events.popleft().synchronize()

    def _finish_plane_round(self) -> None:
        """Round bookkeeping of the xGMI plane: the engine runs serve / pull on its own streams;
        the compute stream waits only for the round the next forward must see."""
        if self.pack_stream is not None:
            # the next round's gradients (PsLinear writes them straight into the buckets during
            # backward) overwrite what this round's packs read: order them after every pack
            torch.cuda.current_stream(self.device).wait_stream(self.pack_stream)
        self.round += 1
        self.stats["rounds"] += 1
        v = max(0, self.round - self.staleness)
        need_round = v - 1
        if need_round >= 0:
            self.plane.wait_pulled(need_round)
        if self.timing:
            self._mark("round_end")
        self.wslot = v % self.nslots
        self.gslot = self.round % self.nslots
        self.pending = [len(b.keys) for b in self.reg.buckets]
        self.launched = [False] * len(self.reg.buckets)
        self._bind(self.wslot, self.gslot)
        self._bound_run_ahead()
        if self.timing:
            self._close_timing_deferred()

    def plane_stats(self, reset: bool = False) -> Dict[str, float]:
        """Per-round means of the xGMI plane engine (serve / pull kernel ms, waits for peers)."""
        return self.plane.stats(reset) if self.plane is not None else {}

    def _close_timing_deferred(self) -> None:
        # keep one step in flight: fold the PREVIOUS step's marks (already complete or nearly)
        # so timing adds no per-step host sync to the critical path
        prev = self._prev_marks
        cur, self._marks = self._marks, []
        if prev:
            self._marks = prev
            self._close_timing()
        self._prev_marks = cur
        self._mark("step0")

    def synchronize(self) -> None:
        """Drain every in-flight round (checkpoint / eval boundary)."""
        if self.plane is not None:
            if self.round > 0:
                self.plane.wait_pulled(self.round - 1)
            return
        if self.gpu:
            while self.round_events:
                torch.cuda.current_stream(self.device).wait_event(self.round_events.popleft())

    # ------------------------------------------------------------------ checkpoint
    def shard_state(self) -> dict:
        """This rank's server shard: fp32 master + optimizer state + clock."""
        self.synchronize()
        return {
            "rank": self.rank, "world": self.world, "round": self.round, "staleness": self.staleness,
            # host SNAPSHOTS (to(copy=True): on a CPU run .cpu() would alias the live shard
            # while a background checkpoint writer is still serialising it)
            "master": [_snap(m) for m in self.master],
            "states": [[[_snap(s) for s in st] for st in sts] for sts in self.states],
            "manifest": {k: {"shape": list(ki.shape), "dtype": str(ki.dtype), "bucket": ki.bucket,
                             "offset": ki.offset, "group": ki.group,
                             "layout": "channels_last" if k in self.cl_keys else "contiguous"}
                         for k, ki in self.reg.keys.items()},
            "buckets": [{"group": b.group, "start": b.start, "size": b.size} for b in self.reg.buckets],
        }

    def load_shard_state(self, st: dict) -> None:
        if st["world"] != self.world or st["rank"] != self.rank:
            raise ValueError("checkpoint was written with a different world size / rank")
        self.synchronize()
        with torch.no_grad():
            for m, src in zip(self.master, st["master"]):
                m.copy_(src.to(m.device))
            for sts, srcs in zip(self.states, st["states"]):
                for s_list, src_list in zip(sts, srcs):
                    for s, src in zip(s_list, src_list):
                        s.copy_(src.to(s.device))
            self.round = int(st["round"])
            # rebuild every replica slot by one pull of the restored masters
            if self.plane is not None:
                self.plane.restore_round(self.round)
                for b, bk in enumerate(self.reg.buckets):
                    lo, hi = bk.owner_range(self.rank)
                    for slot in range(self.nslots):
                        wfull = self.wbuf[bk.group][slot]
                        wfull[lo:hi].copy_(self.master[b].to(wfull.dtype))
                for slot in range(self.nslots):
                    self.plane.gather_all(slot)
            for b, bk in enumerate(self.reg.buckets if self.plane is None else []):
                lo, hi = bk.owner_range(self.rank)
                for slot in range(self.nslots):
                    wfull = self.wbuf[bk.group][slot]
                    wfull[lo:hi].copy_(self.master[b].to(wfull.dtype))
                    # (flat element order, channels_last keys included, is the same on every rank)
                    self.t.all_gather(wfull[bk.start:bk.start + bk.size], wfull[lo:hi])
        self.wslot = max(0, self.round - self.staleness) % self.nslots
        self.gslot = self.round % self.nslots
        for grp in self.gbuf:
            self.gbuf[grp][self.gslot].zero_()
        self._bind(self.wslot, self.gslot)

    def close(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
        if self.plane is not None:
            pl, self.plane = self.plane, None
            try:
                pl.close()
            finally:
                self.t.barrier()
                pl.release()


def _snap(t: torch.Tensor) -> torch.Tensor:
    return t.detach().to("cpu", copy=True)


def _wants_channels_last(p: torch.Tensor) -> bool:
    """Conv weight with spatial extent and >4 input channels held channels_last by the model."""
    return (p.dim() == 4 and p.shape[2] * p.shape[3] > 1 and p.shape[1] > 4
            and p.is_contiguous(memory_format=torch.channels_last) and not p.is_contiguous())


def timed(fn):
    t0 = time.perf_counter()
    fn()
    return (time.perf_counter() - t0) * 1e3
