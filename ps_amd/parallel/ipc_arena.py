"""Device arenas every process of the node can map (the xGMI plane's and the row plane's buffers).

Up to 1 GiB: one hipMalloc'ed block shared by an IPC handle (csrc/plane.cpp ``Arena``).  Above:
physical chunks of at most 1 GiB mapped back to back into one virtual range (``VmmArena``), each
exported as a dma-buf file descriptor -- on this stack hipIpcOpenMemHandle hangs for allocations
above 2 GiB (1.99 GiB opens at once, 2.01 GiB never returns; profiles/r6_plane_ipc_2gib.txt), and a
Llama-3-8B plane arena is ~34 GB.  The descriptors reach the peers over an abstract Unix socket
(SCM_RIGHTS): the exporter serves its fds from a thread, a peer connects, receives them, imports
every chunk and maps them back to back, so both sides see one contiguous arena and the plane
engine's base + offset addressing does not change.
"""
from __future__ import annotations

import os
import socket
import threading
import uuid
from typing import List, Optional

VMM_ABOVE = 1 << 30  # bytes: larger arenas are built from VMM chunks
CHUNK = 1 << 30


def _C():
    from .. import _C as C  # type: ignore

    return C


class IpcArena:
    """``Arena``'s interface (base, tensor(), handle(), open(handle, device), close()) over either
    kind of allocation; the kind follows the size, which every rank computes alike."""

    def __init__(self, nbytes: int, device: int, vmm: Optional[bool] = None, chunk: int = CHUNK):
        P = _C().plane
        self.vmm = nbytes > VMM_ABOVE if vmm is None else bool(vmm)
        self._fds: List[int] = []
        self._srv: Optional[socket.socket] = None
        self._thread: Optional[threading.Thread] = None
        self._stop = threading.Event()
        if not self.vmm:
            self._a = P.Arena(int(nbytes), int(device))
            return
        self._a = P.VmmArena(int(nbytes), int(device), int(chunk))
        self._sizes = [int(s) for s in self._a.chunk_sizes()]
        self._fds = [int(f) for f in self._a.export_fds()]
        self._addr = f"\0psamd_vmm_{uuid.uuid4().hex}"
        self._srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self._srv.bind(self._addr)
        self._srv.listen(64)
        self._srv.settimeout(0.2)
        self._thread = threading.Thread(target=self._serve, daemon=True)
        self._thread.start()

    def _serve(self) -> None:
        while not self._stop.is_set():
            try:
                conn, _ = self._srv.accept()
            except socket.timeout:
                continue
            except OSError:
                return
            with conn:
                socket.send_fds(conn, [b"psamd-vmm"], self._fds)

    @property
    def base(self) -> int:
        return int(self._a.base)

    def tensor(self):
        return self._a.tensor()

    def handle(self):
        """Picklable description a peer's ``open`` takes."""
        if not self.vmm:
            return ("ipc", self._a.handle())
        return ("vmm", self._addr, self._sizes)

    def open(self, h, peer_device: int) -> int:
        """Map a peer's arena into this process; -> its base address here."""
        kind = h[0] if isinstance(h, tuple) else "ipc"
        if kind == "ipc":
            return int(self._a.open(h[1] if isinstance(h, tuple) else h, int(peer_device)))
        _, addr, sizes = h
        with socket.socket(socket.AF_UNIX, socket.SOCK_STREAM) as s:
            s.settimeout(60.0)
            s.connect(addr)
            _, fds, _, _ = socket.recv_fds(s, 64, len(sizes))
        try:
            if len(fds) != len(sizes):
                raise RuntimeError(f"received {len(fds)} chunk descriptors, expected {len(sizes)}")
            return int(self._a.open(list(fds), list(sizes), int(peer_device)))
        finally:
            for f in fds:
                os.close(f)

    def close(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
            self._thread = None
        if self._srv is not None:
            self._srv.close()
            self._srv = None
        for f in self._fds:
            try:
                os.close(f)
            except OSError:
                pass
        self._fds = []
        self._a.close()
