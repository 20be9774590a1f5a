"""Parameter-server clients (reference elephas/parameter/client.py:13-91).

``get_parameters`` returns a list of numpy arrays (the reference's
``np.asarray(list)`` built a ragged object array);
``update_parameters(delta)`` subtracts ``delta`` on the server.  The device
client additionally exposes ``pull_into``/``push_from`` on flat device buffers,
which is what the MI355X workers use on the hot path.
"""
from __future__ import annotations

import abc
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
    """Client of a DeviceServer: same-process (direct) or another process (HIP IPC over xGMI)."""

    client_type = "device"

    def __init__(self, port: int = 4000, server=None, handle=None, like=None):
        self.port = port
        self.server = server
        self.remote = None
        self.like = like
        if handle is not None:
            self.attach(handle)

    def attach(self, handle):
        from ..ops import native
        h, n, locked, lock_name = handle
        self.remote = native.require().RemoteParameterServer(h, n, locked, lock_name)
        self.n = n

    def bind(self, server):
        self.server = server
        self.like = server._like

    def _ps(self):
        if self.server is not None:
            return self.server.ps
        if self.remote is not None:
            return self.remote
        raise RuntimeError("DeviceClient is not bound to a server")

    # flat device-buffer API (hot path)
    def pull_into(self, dst_ptr: int, stream: int) -> None:
        self._ps().pull(dst_ptr, stream)

    def push_from(self, delta_ptr: int, stream: int) -> None:
        self._ps().push(delta_ptr, stream)

    # R lockstep replicas (rows of a [R, n] fp32 buffer, row stride sP elements)
    def pull_replicas(self, P_ptr: int, sP: int, R: int, before_ptr: int, stream: int) -> None:
        """P[r] = theta for every replica and before = theta (one kernel)."""
        self._ps().pull_replicas(P_ptr, sP, R, before_ptr, stream)

    def pull_refresh(self, trainer, before_ptr: int) -> None:
        """Pull fused with the trainer's weight-image refresh: ONE kernel reads theta and
        writes every replica's fp32 master, both bf16 W / W^T parities and `before`."""
        from ..ops import native
        native.require().ps_pull_refresh(self._ps(), trainer.exe, before_ptr, trainer.s)

    def push_replicas(self, P_ptr: int, sP: int, R: int, before_ptr: int, stream: int) -> None:
        """theta -= sum_r (before - P[r]) (one kernel)."""
        self._ps().push_replicas(P_ptr, sP, R, before_ptr, stream)

    # list-of-arrays API (reference compatibility)
    def get_parameters(self):
        if self.server is not None:
            return self.server.get_weights()
        import torch
        from ..ops.plan import unflatten_weights
        buf = torch.empty(self.n, dtype=torch.float32, device="cuda")
        s = torch.cuda.current_stream()
        self.remote.pull(buf.data_ptr(), s.cuda_stream)
        s.synchronize()
        return unflatten_weights(buf.cpu().numpy(), self.like) if self.like else buf.cpu().numpy()

    def update_parameters(self, delta: list):
        import torch
        from ..ops.plan import flatten_weights
        d = torch.from_numpy(flatten_weights(list(delta))).cuda()
        s = torch.cuda.current_stream()
        self.push_from(d.data_ptr(), s.cuda_stream)
        s.synchronize()
