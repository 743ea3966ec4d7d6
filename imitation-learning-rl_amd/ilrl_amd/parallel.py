"""Multi-GPU layout: one process per GPU, env lanes sharded by rank.

* Rank r owns global lanes [off_r, off_r + n_r) (`shard`); each lane's RNG stream is keyed by its GLOBAL id
  (hum_config.lane_offset), so results are independent of how many GPUs share the job.
* Env stepping needs no collective (weak scaling).  The only exchange is the trajectory gather to the
  learner rank (obs / action / reward / done per step or per rollout fragment), done with ONE collective per
  call over torch.distributed ("nccl" = RCCL over xGMI on MI355X, "gloo" on CPU).  The buffers travel as their
  raw bytes (lossless for every dtype), and uneven shards are padded to the largest one and trimmed on arrival.
"""
import ctypes
import math
import os
import queue
import threading
import time

import torch
import torch.distributed as dist


def shard(n_total, world, rank):
    """(lane_offset, n_local) of `rank` for n_total lanes split over `world` ranks (contiguous shards)."""
    base, rem = divmod(n_total, world)
    n = base + (1 if rank < rem else 0)
    off = rank * base + min(rank, rem)
    return off, n


def _row_bytes(t):
    return t[0].numel() * t.element_size() if t.dim() > 1 else t.element_size()


def gather_trajectories(tensors, dst=0, counts=None):
    """Gather per-rank trajectory buffers (same trailing shape and dtype on every rank; leading dim = that
    rank's lanes, may differ between ranks) onto `dst` as one [sum n_r, ...] tensor each, in rank order.

    All buffers are packed, row by row, into ONE uint8 message (their raw bytes: int64 / uint8 / float keep
    their exact values), so RCCL moves one large payload per call: xGMI is point-to-point, so few large
    collectives beat many small ones.  `counts` (every rank's lane count, e.g. from `shard`) skips the count
    exchange.  Returns the list on dst, None elsewhere.  (The benchmark's repeated gather is TrajectoryGather.)"""
    on = dist.is_initialized()   # one rank with the group initialised still runs the collectives (bench --force-dist)
    world = dist.get_world_size() if on else 1
    rank = dist.get_rank() if on else 0
    n = int(tensors[0].shape[0])
    if any(int(t.shape[0]) != n for t in tensors):
        raise ValueError("every buffer needs the same leading (lane) dimension")
    dev = tensors[0].device
    widths = [_row_bytes(t) for t in tensors]
    flat = torch.cat([t.contiguous().reshape(n, -1).view(torch.uint8).reshape(n, w) for t, w in zip(tensors, widths)],
                     dim=1) if n else torch.zeros((0, sum(widths)), dtype=torch.uint8, device=dev)
    if on and dist.get_backend() == "gloo" and flat.is_cuda:   # gloo gathers host tensors
        flat, dev = flat.cpu(), torch.device("cpu")
    if not on:
        full, counts = flat, [n]
    else:
        if counts is None:
            cnt = torch.tensor([n], dtype=torch.int64, device=dev)
            counts_t = [torch.zeros_like(cnt) for _ in range(world)]
            dist.all_gather(counts_t, cnt)
            counts = [int(c.item()) for c in counts_t]
        m = max(counts)
        pad = torch.zeros((m, flat.shape[1]), dtype=torch.uint8, device=dev)
        pad[:n] = flat
        if dist.get_backend() == "nccl":   # RCCL all_gather_into_tensor (RCCL emulates gather with it anyway)
            out = torch.empty((world * m, flat.shape[1]), dtype=torch.uint8, device=dev)
            dist.all_gather_into_tensor(out, pad)
            parts = list(out.split(m, dim=0))
        else:
            parts = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
            dist.gather(pad, gather_list=parts, dst=dst)
        if rank != dst:
            return None
        full = torch.cat([p[:c] for p, c in zip(parts, counts)], dim=0)
    if rank != dst:
        return None
    out, c = [], 0
    for t, w in zip(tensors, widths):
        col = full[:, c:c + w].contiguous()
        out.append(col.view(t.dtype).reshape((full.shape[0],) + tuple(t.shape[1:])))
        c += w
    return out


class TrajectoryGather:
    """The rollout's repeated trajectory gather to the learner rank (reference: RLlib's rollout workers
    ship sample batches to the learner, /root/reference/train_config.py:33-34), built once per run.

    * Static shapes: every rank's lane count is known from the sharding (`counts`, e.g. `shard`), so no count
      exchange and no host synchronisation happen per call.
    * One packed uint8 buffer per fragment, step-major: step t's block (`SB` bytes) holds that step's rows of every
      field for the `m` (largest shard's) lanes - [m, 70] obs, then [m, 17] actions, ... (raw bytes, fields ordered by
      descending item size, each field's rows 8-byte aligned).  So the steps [t0, t1) one env launch produced are ONE
      contiguous byte range, which can travel as soon as that launch is packed (DmaGather's per-launch chunks), and
      `pack` is one hum_pack_rows launch (every field's time-major [k, n, ...] outputs into their rows, the only copy).
    * Asynchronous: `commit(slot, t0, t1, final)` after each pack; the fragment's gather (RCCL point-to-point sends to
      `dst`, `dist.gather`) is issued on the final one, ordered after the packs on the current stream, and returns; the
      next env launches proceed while it moves.  Fragments alternate between `slots` buffers; packing into a slot
      first waits for that slot's previous gather.
    * `result` presents the gathered fragment lane-major, {field: [sum n_r, G, ...]} (RLlib's per-env rows).
    * gloo (CPU tests): the same layout, gathered synchronously through host memory.
    """

    def __init__(self, fields, counts, G, device, dst=0, slots=2):
        self.on = dist.is_initialized()
        self.world = dist.get_world_size() if self.on else 1
        self.rank = dist.get_rank() if self.on else 0
        if len(counts) != self.world:
            raise ValueError("counts: one lane count per rank")
        self.counts, self.G, self.dst, self.dev = [int(c) for c in counts], int(G), dst, torch.device(device)
        self.n, self.m = self.counts[self.rank], max(self.counts)
        self.nccl = self.on and dist.get_backend() == "nccl"
        self.fields = []   # (name, per-step trailing shape, dtype, byte offset in the step block, bytes per lane-step)
        off = 0
        for name, shape, dtype in sorted(fields, key=lambda f: -torch.empty(0, dtype=f[2]).element_size()):
            isz = torch.empty(0, dtype=dtype).element_size()
            w = int(math.prod(shape)) * isz
            self.fields.append((name, tuple(shape), dtype, off, w))
            off += -(-(self.m * w) // 8) * 8
        self.order = [f[0] for f in fields]
        self.SB = off                 # bytes per step block (a multiple of 8)
        self.W = sum(f[4] for f in self.fields)   # payload bytes per lane-step
        self.bytes = self.G * self.SB
        self.send = [torch.zeros(self.bytes, dtype=torch.uint8, device=self.dev) for _ in range(slots)]
        self.recv = [[torch.empty(self.bytes, dtype=torch.uint8, device=self.dev if self.nccl else "cpu")
                      for _ in range(self.world)] if self.rank == dst else None for _ in range(slots)]
        self.work = [None] * slots
        self.fragments = 0

    def _view(self, buf, name, rows=None):
        """Time-major typed view [G, rows (default m), ...] of one field in a fragment buffer."""
        for nm, shape, dtype, off, w in self.fields:
            if nm == name:
                v = buf.view(self.G, self.SB)[:, off:off + self.m * w].view(dtype).unflatten(1, (self.m,) + shape)
                return v[:, :rows] if rows is not None else v
        raise KeyError(name)

    def pack(self, slot, t0, outputs):
        """outputs: {field: [k, n, ...] time-major tensor of steps t0 .. t0 + k - 1 of the fragment}.  On the device
        one hum_pack_rows launch copies every field (the HIP library's packing kernel); on the host, torch copies.
        Every field must hold the same k steps and 0 <= t0, t0 + k <= G: the packing kernel writes rows by offset and
        knows nothing of the fragment's capacity, so a crossing pack is refused here on both paths."""
        t0 = int(t0)
        ks = {int(x.shape[0]) for x in outputs.values()}
        if len(ks) != 1:
            raise ValueError("pack: every field needs the same leading step count, got %s" % sorted(ks))
        k = ks.pop()
        if t0 < 0 or t0 + k > self.G:
            raise ValueError("pack: steps [%d, %d) cross the fragment of %d steps" % (t0, t0 + k, self.G))
        self._wait_slot(slot, t0)
        if self.dev.type == "cuda":
            return self._pack_native(slot, t0, outputs)
        for name, x in outputs.items():
            self._view(self.send[slot], name, self.n)[t0:t0 + x.shape[0]].copy_(x)

    def _wait_slot(self, slot, t0):
        if self.work[slot] is not None:   # the slot's previous gather must have read the buffer
            self.work[slot].wait()
            self.work[slot] = None

    def _pack_native(self, slot, t0, outputs):
        import ctypes
        from . import _native as N
        kk = None
        arr = (N.HumPackField * len(outputs))()
        base = self.send[slot].data_ptr()
        for j, (name, x) in enumerate(outputs.items()):
            nm, shape, dtype, off, w = next(f for f in self.fields if f[0] == name)
            if x.dtype != dtype or tuple(x.shape[2:]) != shape or x.shape[1] != self.n or x.stride(-1) != 1 and w > x.element_size():
                raise ValueError("pack: field %s has shape %s / dtype %s" % (name, tuple(x.shape), x.dtype))
            if kk is None:
                kk = int(x.shape[0])
            isz = x.element_size()
            arr[j].src, arr[j].dst = x.data_ptr(), base + off
            arr[j].src_step, arr[j].src_lane = x.stride(0) * isz, x.stride(1) * isz
            arr[j].dst_step, arr[j].dst_lane, arr[j].row_bytes = self.SB, w, w
        stream = torch.cuda.current_stream(self.dev).cuda_stream
        N.check(N.lib().hum_pack_rows(arr, len(outputs), kk, self.n, t0, ctypes.c_void_p(stream)), "hum_pack_rows")

    def commit(self, slot, t0, t1, final):
        """Steps [t0, t1) of slot's fragment are packed; `final`: the fragment is complete (or the run ends) - gather
        it.  (The collective transport moves whole fragments; DmaGather moves every committed range at once.)"""
        if final:
            self.start(slot)

    def start(self, slot):
        """Gather slot's packed fragment onto dst (asynchronous on RCCL)."""
        self.fragments += 1
        if not self.on:
            if self.recv[slot] is not None:
                self.recv[slot][0].copy_(self.send[slot])
            return
        if self.nccl:
            self.work[slot] = dist.gather(self.send[slot], gather_list=self.recv[slot], dst=self.dst, async_op=True)
        else:   # gloo gathers host tensors
            dist.gather(self.send[slot].cpu(), gather_list=self.recv[slot], dst=self.dst)

    def wait(self, slot=None):
        for j in range(len(self.work)) if slot is None else [slot]:
            if self.work[j] is not None:
                self.work[j].wait()
                self.work[j] = None

    def result(self, slot):
        """dst: the gathered fragment lane-major, {field: [sum n_r, G, ...]} in rank order (after wait); None
        elsewhere."""
        if self.recv[slot] is None:
            return None
        return {nm: torch.cat([self._view(r, nm, c) for r, c in zip(self.recv[slot], self.counts)],
                              dim=1).transpose(0, 1).contiguous() for nm in self.order}


class DmaUnavailable(RuntimeError):
    """Raised on EVERY rank (after a collective agreement) when the copy-engine transport cannot be set up on one of
    them - an IPC export / mapping or the probe pull failed - so callers can fall back to the collective transport
    consistently."""


class DmaGather(TrajectoryGather):
    """TrajectoryGather whose fragments travel on the SDMA copy engines instead of a collective's kernels (SURVEY
    8(e); VERDICT round 5: the env kernel holds every CU's registers and LDS for a launch's whole duration, so an RCCL
    send / recv kernel - or a blit copy - cannot run beside it, while a copy engine can: tools/micro/overlap.py).

    * Setup (collective, once): every rank exports its `slots` packed send buffers (hum_ipc_export); the handles are
      all-gathered over a gloo control group; the learner rank maps every peer's buffers (hum_ipc_open).
    * Per env launch (a chunk): pack as TrajectoryGather (one hum_pack_rows launch), then `commit` records an event
      on the packing stream and hands the chunk - the launch's steps [t0, t1), one contiguous byte range of the
      step-major fragment - to a helper thread; the main thread goes on launching.  A sender's helper waits for its
      event, tells the learner "chunk c is packed" over the control group and waits for the learner's "pulled"; the
      learner's helper waits for its own event, then for each sender's "packed" issues an SDMA pull of that sender's
      range (hum_dma_copy; engines round-robin), waits for all of them and answers "pulled".  So a launch's rows move
      while the next launch computes, and what is still in flight when the last launch ends is that launch's rows
      only (bench.py ends a gathering run with a short drain launch).  A slot is packed again (t0 = 0) only after
      its previous fragment's last chunk was pulled.
    * The control messages are 8-byte host tensors on their own gloo group, used by the helper threads only.
    Same layout and result() as TrajectoryGather; `transport` names it in the bench line."""

    transport = "dma"

    def __init__(self, fields, counts, G, device, dst=0, slots=2):
        super().__init__(fields, counts, G, device, dst=dst, slots=slots)
        if not (self.on and self.dev.type == "cuda"):
            raise ValueError("DmaGather needs an initialised process group and device buffers")
        if self.rank == dst:   # the learner's receive buffers live on its device whatever the default group's backend
            self.recv = [[torch.empty(self.bytes, dtype=torch.uint8, device=self.dev) for _ in range(self.world)]
                         for _ in range(slots)]
        from . import _native as N
        self.N = N
        L = N.lib()
        self.ctrl = dist.new_group(backend="gloo")
        mine = []
        for b in self.send:
            h = ctypes.create_string_buffer(N.HUM_IPC_HANDLE_BYTES)
            off = ctypes.c_uint64(0)
            N.check(L.hum_ipc_export(ctypes.c_void_p(b.data_ptr()), h, ctypes.byref(off)), "hum_ipc_export")
            mine.append((h.raw, int(off.value)))
        allh = [None] * self.world
        dist.all_gather_object(allh, mine, group=self.ctrl)
        self.remote = None   # learner: remote[r][slot] = (mapped pointer, mapping base)
        err = ""
        if self.rank == dst:
            self.remote = {}
            try:
                for r in range(self.world):
                    if r == dst:
                        continue
                    self.remote[r] = []
                    for hb, off in allh[r]:
                        p = ctypes.c_void_p()
                        N.check(L.hum_ipc_open(hb, off, ctypes.byref(p)), "hum_ipc_open")
                        self.remote[r].append((p.value, p.value - off))
                if os.environ.get("ILRL_AMD_DMA_PROBE_FAIL") == "1":   # tests: the fallback path
                    raise RuntimeError("injected probe failure (ILRL_AMD_DMA_PROBE_FAIL)")
                # probe: one small pull from every mapped slot (and the own one) on the copy engines
                for r in range(self.world):
                    for j in range(slots):
                        src = self.send[j].data_ptr() if r == dst else self.remote[r][j][0]
                        t = N.HumDmaTicket()
                        N.check(L.hum_dma_copy(ctypes.c_void_p(self.recv[j][r].data_ptr()), ctypes.c_void_p(src),
                                               min(256, self.bytes), r, ctypes.byref(t)), "hum_dma_copy")
                        N.check(L.hum_dma_wait(ctypes.byref(t)), "hum_dma_wait")
            except Exception as e:   # noqa: BLE001 - reported to every rank below
                err = repr(e)
        errs = [None] * self.world
        dist.all_gather_object(errs, err, group=self.ctrl)
        bad = [e for e in errs if e]
        if bad:
            self._unmap()
            raise DmaUnavailable("copy-engine transport unavailable: %s" % bad[0])
        self.free = [threading.Event() for _ in range(slots)]   # the slot's last fragment has been pulled
        for e in self.free:
            e.set()
        self.chunks = 0
        self.trace = [] if os.environ.get("ILRL_DMA_TRACE") == "1" else None   # diagnostics: per-chunk timestamps
        self.jobs = queue.Queue()
        self.err = []
        self.thread = threading.Thread(target=self._helper, name="dma-gather", daemon=True)
        self.thread.start()

    def _wait_slot(self, slot, t0):
        if t0 == 0 and not self.free[slot].is_set():   # a new fragment: the slot's previous one must be pulled
            self._wait_free(slot)

    def _wait_free(self, slot):
        while not self.free[slot].wait(0.05):
            if self.err:
                raise RuntimeError("DmaGather helper failed: %s" % self.err[0])

    def commit(self, slot, t0, t1, final):
        if not 0 <= t0 < t1 <= self.G:
            raise ValueError("commit: steps [%d, %d) outside the fragment of %d steps" % (t0, t1, self.G))
        if t0 == 0:
            self.free[slot].clear()
        if final:
            self.fragments += 1
        self.chunks += 1
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        if self.trace is not None:
            self.trace.append(("commit", self.chunks, time.perf_counter()))
        self.jobs.put((self.chunks, slot, t0, t1, final, ev))

    def start(self, slot):
        """The whole fragment as one chunk."""
        self.commit(slot, 0, self.G, True)

    def wait(self, slot=None):
        for j in range(len(self.free)) if slot is None else [slot]:
            self._wait_free(j)

    def _helper(self):
        """The transfer loop (one chunk per job).  A failure on any rank is passed on as a negative message, so
        every rank's helper stops and its main thread raises from pack / wait instead of waiting forever."""
        L = self.N.lib()
        msg = torch.zeros(1, dtype=torch.int64)
        send = lambda v, r: dist.send(torch.tensor([v], dtype=torch.int64), r, group=self.ctrl)
        try:
            while True:
                job = self.jobs.get()
                if job is None:
                    return
                c, slot, t0, t1, final, ev = job
                lo, nbytes = t0 * self.SB, (t1 - t0) * self.SB
                if self.rank != self.dst:
                    try:
                        ev.synchronize()
                    except Exception:
                        send(-1, self.dst)
                        raise
                    send(c, self.dst)                           # packed
                    dist.recv(msg, self.dst, group=self.ctrl)   # pulled
                    if int(msg.item()) != c:
                        raise RuntimeError("chunk %d: the learner answered %d" % (c, int(msg.item())))
                else:
                    tickets, posted = [], {}
                    tr = self.trace
                    try:
                        # every sender's "packed" is posted at once (the senders finish the launch together: the
                        # waits overlap instead of adding up), then each pull is issued as its message is in
                        peers = [r for r in range(self.world) if r != self.dst]
                        msgs = {r: torch.zeros(1, dtype=torch.int64) for r in peers}
                        posted = {r: dist.irecv(msgs[r], r, group=self.ctrl) for r in peers}
                        ev.synchronize()
                        if tr is not None:
                            tr.append(("packed", c, time.perf_counter()))
                        for r in [self.dst] + peers:
                            if r == self.dst:   # its own rows: also a copy-engine transfer
                                src_ptr = self.send[slot].data_ptr()
                            else:
                                posted.pop(r).wait()
                                if int(msgs[r].item()) != c:
                                    raise RuntimeError("rank %d sent %d for chunk %d" % (r, int(msgs[r].item()), c))
                                src_ptr = self.remote[r][slot][0]
                            if self.counts[r]:
                                t = self.N.HumDmaTicket()
                                self.N.check(L.hum_dma_copy(ctypes.c_void_p(self.recv[slot][r].data_ptr() + lo),
                                                            ctypes.c_void_p(src_ptr + lo), nbytes, len(tickets),
                                                            ctypes.byref(t)), "hum_dma_copy")
                                tickets.append(t)
                        if tr is not None:
                            tr.append(("issued", c, time.perf_counter()))
                        while tickets:
                            self.N.check(L.hum_dma_wait(ctypes.byref(tickets.pop(0))), "hum_dma_wait")
                        if tr is not None:
                            tr.append(("pulled", c, time.perf_counter()))
                    except Exception:
                        for t in tickets:   # retire the copies in flight before giving up
                            L.hum_dma_wait(ctypes.byref(t))
                        for w in posted.values():   # the senders' messages still posted
                            w.wait()
                        for r in range(self.world):
                            if r != self.dst:
                                send(-1, r)
                        raise
                    done = torch.tensor([c], dtype=torch.int64)
                    for w in [dist.isend(done, r, group=self.ctrl) for r in range(self.world) if r != self.dst]:
                        w.wait()                                # pulled
                if final:
                    self.free[slot].set()
        except Exception as e:   # surfaced on the main thread by pack / wait
            self.err.append(repr(e))

    def close(self):
        """Drain the helper, unmap the peers' buffers, and keep every exporter's buffers alive until the learner has
        unmapped them (a barrier on the control group)."""
        self.wait()
        self.jobs.put(None)
        self.thread.join()
        self._unmap()
        dist.barrier(group=self.ctrl)

    def _unmap(self):
        if self.remote:
            L = self.N.lib()
            for r, lst in self.remote.items():
                for _, base in lst:
                    L.hum_ipc_close(ctypes.c_void_p(base))
            self.remote = None
