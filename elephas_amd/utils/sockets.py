"""Master discovery and length-prefixed socket framing
(reference elephas/utils/sockets.py:6-71: 20-byte zero-padded ASCII length +
payload).  The payload is NOT pickle (reference quirk SURVEY.md §2.8 item 10:
unauthenticated pickle = remote code execution): it is a numpy ``.npz``
archive loaded with ``allow_pickle=False``."""
import io
import os
from socket import gethostbyname, gethostname
from typing import Any

import numpy as np


def determine_master(port: int = 4000) -> str:
    host = os.environ.get("SPARK_LOCAL_IP") or os.environ.get("ELEPHAS_AMD_PS_HOST")
    if not host:
        try:
            host = gethostbyname(gethostname())
        except OSError:
            host = "127.0.0.1"
    return f"{host}:{port}"


def encode(obj: Any) -> bytes:
    """list of arrays -> .npz bytes; dict {'delta': [...]} supported."""
    buf = io.BytesIO()
    if isinstance(obj, dict):
        key, arrays = next(iter(obj.items()))
        np.savez(buf, __key__=np.array(key), **{f"a{i}": np.asarray(a) for i, a in enumerate(arrays)})
    else:
        np.savez(buf, **{f"a{i}": np.asarray(a) for i, a in enumerate(obj)})
    return buf.getvalue()


def decode(data: bytes) -> Any:
    with np.load(io.BytesIO(data), allow_pickle=False) as z:
        names = sorted((k for k in z.files if k.startswith("a")), key=lambda k: int(k[1:]))
        arrays = [z[k] for k in names]
        if "__key__" in z.files:
            return {str(z["__key__"]): arrays}
        return arrays


def _receive_all(socket, num_bytes: int) -> bytes:
    buffer = bytearray()
    while len(buffer) < num_bytes:
        chunk = socket.recv(min(num_bytes - len(buffer), 1 << 20))
        if not chunk:
            raise ConnectionError("socket closed while receiving")
        buffer += chunk
    return bytes(buffer)


def receive(socket, num_bytes: int = 20) -> Any:
    length = int(_receive_all(socket, num_bytes).decode())
    return decode(_receive_all(socket, length))


def send(socket, data: Any, num_bytes: int = 20) -> None:
    payload = encode(data)
    length = str(len(payload)).zfill(num_bytes).encode()
    socket.sendall(length + payload)
