"""Parameter-server clients (reference elephas/parameter/client.py:13-91).

``get_parameters`` returns a list of numpy arrays (the reference's
``np.asarray(list)`` built a ragged object array);
``update_parameters(delta)`` subtracts ``delta`` on the server.  The device
client additionally exposes ``pull_into``/``push_from`` on flat device buffers,
which is what the MI355X workers use on the hot path.
"""
from __future__ import annotations

import abc
import os
import socket
import urllib.request as urllib2
from typing import List

import numpy as np

from ..utils.sockets import decode, determine_master, encode, receive, send


class BaseParameterClient(abc.ABC):
    client_type = "base"

    @classmethod
    def get_client(cls, client_type: str, port: int = 4000):
        try:
            return next(cl for cl in cls.__subclasses__() if cl.client_type == client_type)(port)
        except StopIteration:
            raise ValueError("Parameter server mode has to be either `http`, `socket` or `device`, "
                             "got {}".format(client_type))

    @abc.abstractmethod
    def update_parameters(self, delta: list):
        raise NotImplementedError

    @abc.abstractmethod
    def get_parameters(self):
        raise NotImplementedError


class HttpClient(BaseParameterClient):
    client_type = "http"

    def __init__(self, port: int = 4000):
        self.master_url = determine_master(port=port)
        self.headers = {"Content-Type": "application/elephas"}

    def get_parameters(self) -> List[np.ndarray]:
        request = urllib2.Request(f"http://{self.master_url}/parameters", headers=self.headers)
        return decode(urllib2.urlopen(request).read())

    def update_parameters(self, delta: list):
        request = urllib2.Request(f"http://{self.master_url}/update", encode(list(delta)), headers=self.headers)
        return urllib2.urlopen(request).read()


class SocketClient(BaseParameterClient):
    client_type = "socket"

    def __init__(self, port: int = 4000):
        self.port = port

    def _connect(self):
        host = determine_master(port=self.port).split(":")[0]
        sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        sock.connect((host, self.port))
        return sock

    def get_parameters(self) -> List[np.ndarray]:
        with self._connect() as sock:
            sock.sendall(b"g")
            return receive(sock)

    def update_parameters(self, delta: list):
        with self._connect() as sock:
            sock.sendall(b"u")
            send(sock, {"delta": list(delta)})


class DeviceClient(BaseParameterClient):
    """This rank's endpoint of the sharded device parameter server.

    ``connect`` is collective over the job's ranks (every rank allocates its shard
    and maps every other rank's through HIP IPC); afterwards every call enqueues
    kernels on the given stream and returns without synchronising it.
    """

    client_type = "device"

    def __init__(self, port: int = 4000, like=None):
        self.port = port
        self.like = like
        self.ps = None
        self.n = None

    def connect(self, n: int, mode: str, server=None, rank: int = None, world: int = None, device: int = None,
                allgather=None, chunk: int = 4096):
        import torch
        from ..ops import native
        from ..parallel import dist
        from ..parallel.p2p import exchange_handles
        rank = dist.rank() if rank is None else rank
        world = dist.world_size() if world is None else world
        device = torch.cuda.current_device() if device is None else device
        consistent = 1 if mode == "asynchronous" else 0
        self.ps = native.require().ShardedParameterServer(rank, world, int(n), consistent, device, chunk)
        self.ps.open(exchange_handles(self.ps.handle(), allgather))
        self.n = int(n)
        self.chunk = int(chunk)
        if world > 1 and os.environ.get("ELEPHAS_AMD_PS_SELFTEST", "1") != "0":
            self.self_test(rank, world, bool(consistent), allgather or dist.all_gather_object)
        if server is not None:
            server.native = self.ps
            self.like = server._like
        return self

    def self_test(self, rank: int, world: int, consistent: bool, allgather, K: int = 6) -> dict:
        """Collective check of the sharded PS on the actual interconnect before any worker
        uses it (remote fp32 atomics into peer-mapped uncached memory, flag ordering
        across devices): every rank pushes K integer-valued deltas at once while pulling
        snapshots; the final theta must be the exact sum of every push, no wait may time
        out, and (asynchronous mode) no snapshot may hold a torn chunk -- a chunk is
        constant in the pattern, so a consistent pull sees every element of it from
        the same set of pushes.  Voted: every rank raises if any rank failed.
        theta is left at zero; the caller sets the initial weights afterwards."""
        import torch
        from ..parallel import fault
        n, ch = self.n, self.chunk
        dev = torch.device("cuda", torch.cuda.current_device())
        s = torch.cuda.current_stream(dev)
        zero = torch.zeros(n, dtype=torch.float32, device=dev)
        if rank == 0:
            torch.cuda.synchronize(dev)
            self.ps.set(zero.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize(dev)
        allgather(None)   # theta = 0 before any push
        pat = (torch.arange(n, device=dev) // ch % 5 + 1).to(torch.float32)
        delta = pat * -float(rank + 1)   # push does theta -= delta
        try:
            fault.maybe_inject("ps_selftest", rank)
        except fault.InjectedFault:
            delta = delta * 2.0           # a wrong contribution the vote must catch
        nsnap = K if n <= (4 << 20) else 2
        # rows padded to 16 bytes: pull writes 16-byte vectors
        snaps = torch.empty(nsnap, (n + 3) // 4 * 4, dtype=torch.float32, device=dev)[:, :n]
        sp, sq = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        sp.wait_stream(s)
        sq.wait_stream(s)
        for k in range(K):
            self.ps.push_delta(delta.data_ptr(), sp.cuda_stream)
            if k < nsnap:
                self.ps.pull(snaps[k].data_ptr(), sq.cuda_stream)
        torch.cuda.synchronize(dev)
        allgather(None)   # every rank's pushes have landed
        fin = torch.empty(n, dtype=torch.float32, device=dev)
        self.ps.pull(fin.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize(dev)
        want = pat * float(K * world * (world + 1) // 2)
        res = {"exact": bool(torch.equal(fin, want)), "error": int(self.ps.error()), "torn_chunks": 0}
        if consistent:
            pad = (-n) % ch
            blk = torch.nn.functional.pad(snaps, (0, pad)).reshape(nsnap, -1, ch)
            edge = blk[:, :, :1].expand_as(blk).clone()
            if pad:   # the padded tail of the last chunk compares against itself
                blk[:, -1, ch - pad:] = edge[:, -1, ch - pad:]
            res["torn_chunks"] = int((blk != edge).any(2).sum())
        if rank == 0:
            self.ps.set(zero.data_ptr(), s.cuda_stream)
            torch.cuda.synchronize(dev)
        votes = allgather(res)
        self.self_test_result = votes
        bad = [(r, v) for r, v in enumerate(votes) if not v["exact"] or v["error"] or v["torn_chunks"]]
        if bad:
            raise RuntimeError(
                "device parameter server self-test failed on the peer interconnect "
                f"(rank, result): {bad}; the sharded HBM parameter server cannot be trusted on this "
                "node -- use parameter_server_mode='http' or 'socket', or mode='synchronous'")
        return res

    def close(self, release: bool = False):
        """Drop this rank's endpoint.  ``release``: the caller guarantees every rank has
        finished every pull / push (e.g. after a collective that follows the final
        stream synchronisation), so this rank's shard can be freed; otherwise it stays
        allocated until process exit (freeing memory a peer may still be reading faults
        the reader)."""
        if self.ps is not None and release:
            self.ps.release()
        self.ps = None

    def _native(self):
        if self.ps is None:
            raise RuntimeError("DeviceClient is not connected (DeviceClient.connect is collective)")
        return self.ps

    # flat device-buffer API (hot path; stream-ordered, no host synchronisation)
    def pull_into(self, dst_ptr: int, stream: int) -> None:
        self._native().pull(dst_ptr, stream)

    def pull_into_replicas(self, dst_ptr: int, P_ptr: int, sP: int, R: int, stream: int) -> None:
        """dst = theta and every replica row P[r] = theta, one gather kernel."""
        self._native().pull_replicas(dst_ptr, P_ptr, sP, R, stream)

    def push_from(self, delta_ptr: int, stream: int) -> None:
        """theta -= delta (the reference's update semantics)."""
        self._native().push_delta(delta_ptr, stream)

    def pull_refresh(self, trainer, before_ptr: int) -> None:
        """before = theta (one gather kernel), then every replica's fp32 master and both
        weight-image parities from it (one kernel)."""
        self._native().pull(before_ptr, trainer.s)
        trainer.exe.refresh_from(before_ptr, 0, trainer.s)

    def push_replicas(self, P_ptr: int, sP: int, R: int, before_ptr: int, stream: int) -> None:
        """theta += sum_r (P[r] - before) (one kernel)."""
        self._native().push_replicas(P_ptr, sP, R, before_ptr, stream)

    def check(self) -> None:
        e = self._native().error()
        if e:
            raise RuntimeError(f"device parameter server: a wait timed out (error word {e})")

    # list-of-arrays API (reference compatibility; synchronous)
    def get_parameters(self):
        import torch
        from ..ops.plan import unflatten_weights
        buf = torch.empty(self.n, dtype=torch.float32, device="cuda")
        s = torch.cuda.current_stream()
        self.pull_into(buf.data_ptr(), s.cuda_stream)
        s.synchronize()
        return unflatten_weights(buf.cpu().numpy(), self.like) if self.like else buf.cpu().numpy()

    def update_parameters(self, delta: list):
        import torch
        from ..ops.plan import flatten_weights
        d = torch.from_numpy(flatten_weights(list(delta))).cuda()
        s = torch.cuda.current_stream()
        self.push_from(d.data_ptr(), s.cuda_stream)
        s.synchronize()
