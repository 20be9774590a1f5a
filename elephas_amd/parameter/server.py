"""Parameter servers for the asynchronous / hogwild training modes.

Three transports behind the reference's server API
(reference elephas/parameter/server.py:17-233):
  * ``DeviceServer``  (MI355X-native, default on GPU): the master parameters
    are one flat fp32 vector sharded in 4096-parameter chunks over the GPUs of
    the job (``_C.ShardedParameterServer``, csrc/kernels/peer.hip); every rank
    maps every shard through HIP IPC.  A pull is one gather kernel, a push one
    kernel of fp32 atomic adds into the owners' memory over xGMI -- no host
    lock, no stream synchronisation, capturable in a hipGraph.  Pushes are
    never lost in either mode; 'asynchronous' pulls are chunk-consistent (a
    pulled chunk never holds half of a push, per-chunk began/ended counters),
    'hogwild' pulls read whatever is there.
  * ``HttpServer`` / ``SocketServer`` (host, cross-process compat transports
    with the reference's routes and opcodes).  Payloads are ``.npz`` archives
    read with ``allow_pickle=False`` instead of pickle.
Fixes of reference quirks: servers restart cleanly for a
second ``fit`` (item 3), the socket server reads weights under the write lock
(item 4) and its listener exits when the peer closes (item 4).
"""
from __future__ import annotations

import abc
import io
import logging
import socket
import threading
from typing import List, Optional

import numpy as np

from ..utils.functional_utils import subtract_params
from ..utils.notebook_utils import is_running_in_notebook
from ..utils.rwlock import RWLock as Lock
from ..utils.serialization import dict_to_model
from ..utils.sockets import decode, determine_master, encode, receive, send

log = logging.getLogger("elephas_amd")


class BaseParameterServer(abc.ABC):
    def __init__(self, model, port: int, mode: str, **kwargs):
        self.port = port
        self.mode = mode
        self.custom_objects = kwargs.get("custom_objects")
        self.master_network = dict_to_model(model, self.custom_objects)

    @abc.abstractmethod
    def start(self):
        raise NotImplementedError

    @abc.abstractmethod
    def stop(self):
        raise NotImplementedError

    # host-side accessors (all transports)
    def get_weights(self) -> List[np.ndarray]:
        return self.master_network.get_weights()

    def set_weights(self, weights) -> None:
        self.master_network.set_weights(weights)


class HttpServer(BaseParameterServer):
    """Flask server with ``/``, ``GET /parameters`` and ``POST /update`` (threaded werkzeug)."""

    def __init__(self, model, port: int, mode: str, **kwargs):
        super().__init__(model, port, mode, **kwargs)
        self.master_url = None
        if is_running_in_notebook():
            self.threaded, self.use_reloader, self.debug = False, False, False
        else:
            self.debug = kwargs.get("debug", False)
            self.threaded = kwargs.get("threaded", True)
            self.use_reloader = False
        self.lock = Lock()
        self.weights = self.master_network.get_weights()
        self._srv = None
        self._thread = None

    def get_weights(self):
        return [w.copy() for w in self.weights]

    def set_weights(self, weights):
        self.lock.acquire_write()
        self.weights = [np.asarray(w, np.float32).copy() for w in weights]
        self.lock.release()

    def _app(self):
        from flask import Flask, request
        app = Flask(__name__)

        @app.route("/")
        def home():
            return "Elephas"

        @app.route("/parameters", methods=["GET"])
        def handle_get_parameters():
            if self.mode == "asynchronous":
                self.lock.acquire_read()
            try:
                payload = encode(self.weights)
            finally:
                if self.mode == "asynchronous":
                    self.lock.release()
            return payload

        @app.route("/update", methods=["POST"])
        def handle_update_parameters():
            delta = decode(request.data)
            if self.mode == "asynchronous":
                self.lock.acquire_write()
            try:
                self.weights = subtract_params(self.weights, delta)
            finally:
                if self.mode == "asynchronous":
                    self.lock.release()
            return "Update done"

        return app

    def start(self):
        if self._srv is not None:
            self.stop()
        from werkzeug.serving import make_server
        host = determine_master(self.port).split(":")[0]
        logging.getLogger("werkzeug").setLevel(logging.ERROR)
        self._srv = make_server(host, self.port, self._app(), threaded=self.threaded)
        self._thread = threading.Thread(target=self._srv.serve_forever, daemon=True)
        self._thread.start()
        self.master_url = determine_master(self.port)

    def stop(self):
        if self._srv is not None:
            self._srv.shutdown()
            self._srv.server_close()
            self._thread.join()
            self._srv, self._thread = None, None


class SocketServer(BaseParameterServer):
    """Raw TCP server: 1-byte opcode ``g``/``u`` + 20-byte length + payload."""

    def __init__(self, model, port: int, mode: str, **kwargs):
        super().__init__(model, port, mode, **kwargs)
        self.socket = None
        self.runs = False
        self.connections = []
        self.lock = Lock()
        self.thread = None
        self._ready = threading.Event()

    def start(self):
        if self.thread is not None:
            self.stop()
        self._ready.clear()
        self.thread = threading.Thread(target=self.start_server, daemon=True)
        self.thread.start()
        self._ready.wait(10)

    def stop(self):
        self.stop_server()
        if self.thread is not None:
            self.thread.join()
        self.thread = None

    def start_server(self):
        sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        host = determine_master(port=self.port).split(":")[0]
        sock.bind((host, self.port))
        sock.listen(16)
        self.socket = sock
        self.runs = True
        self._ready.set()
        self.run()

    def stop_server(self):
        self.runs = False
        if self.socket:
            try:
                host = determine_master(port=self.port).split(":")[0]
                with socket.create_connection((host, self.port), timeout=1):
                    pass
            except OSError:
                pass
            for t in self.connections:
                t.join(timeout=5)
            self.socket.close()
        self.socket = None
        self.connections = []

    def update_parameters(self, conn):
        data = receive(conn)
        delta = data["delta"]
        if self.mode == "asynchronous":
            self.lock.acquire_write()
        try:
            weights = self.master_network.get_weights()
            self.master_network.set_weights(subtract_params(weights, delta))
        finally:
            if self.mode == "asynchronous":
                self.lock.release()

    def get_parameters(self, conn):
        if self.mode == "asynchronous":
            self.lock.acquire_read()
        try:
            weights = self.master_network.get_weights()
        finally:
            if self.mode == "asynchronous":
                self.lock.release()
        send(conn, weights)

    def action_listener(self, conn):
        with conn:
            while self.runs:
                op = conn.recv(1)
                if not op:
                    return
                op = op.decode()
                if op == "u":
                    self.update_parameters(conn)
                elif op == "g":
                    self.get_parameters(conn)

    def run(self):
        while self.runs:
            try:
                conn, addr = self.socket.accept()
            except OSError:
                return
            if not self.runs:
                conn.close()
                return
            t = threading.Thread(target=self.action_listener, args=(conn,), daemon=True)
            t.start()
            self.connections.append(t)


class DeviceServer(BaseParameterServer):
    """Rank 0's handle on the sharded HBM parameter server (see module doc).

    The native state (``_C.ShardedParameterServer``: theta cut into chunks spread
    over every rank's GPU memory) is created collectively by ``DeviceClient.connect``
    on every rank when a fit starts; before that the server holds the weights on
    the host like the other transports.
    """

    def __init__(self, model, port: int, mode: str, **kwargs):
        super().__init__(model, port, mode, **kwargs)
        self._like = self.master_network.get_weights()
        self.n = int(sum(w.size for w in self._like))
        self.native = None      # this rank's ShardedParameterServer once connected
        self.running = False

    def start(self):
        self.running = True

    def stop(self):
        self.running = False

    def close(self):
        self.native = None

    def set_weights(self, weights):
        if self.native is None:
            self.master_network.set_weights(weights)
            return
        import torch
        from ..ops.plan import flatten_weights
        flat = torch.from_numpy(flatten_weights(list(weights))).cuda()
        s = torch.cuda.current_stream()
        self.native.set(flat.data_ptr(), s.cuda_stream)
        s.synchronize()

    def get_weights(self):
        if self.native is None:
            return self.master_network.get_weights()
        import torch
        from ..ops.plan import unflatten_weights
        buf = torch.empty(self.n, dtype=torch.float32, device="cuda")
        s = torch.cuda.current_stream()
        self.native.pull(buf.data_ptr(), s.cuda_stream)
        s.synchronize()
        return unflatten_weights(buf.cpu().numpy(), self._like)
