"""Admin REST API (chana-mq-server/.../rest/AdminApi.scala:20-61, AMQPServer.scala:94-133).

Routes (bound to localhost only, like the reference):
  GET /admin/vhost/put/{vhost}[/]     -> create vhost      (200 on completion, 500 on failure)
  GET /admin/vhost/delete/{vhost}[/]  -> delete vhost (no cascade, parity: SURVEY A.Q28)
Superset:
  GET /admin/stats  GET /admin/queues  GET /admin/health
Every response carries ``Access-Control-Allow-Origin: *`` and is access-logged with
method, uri, status, elapsed ms and bytes (AMQPServer.scala:114-133).
"""

import logging
import re
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

log = logging.getLogger("chanamq.admin")

_VHOST = re.compile(r"^/admin/vhost/(put|delete)/([^/]+)/?$")


def make_handler(broker, extra=None):
    class Handler(BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def _reply(self, status, body=b"", ctype="text/plain"):
            self.send_response(status)
            self.send_header("Access-Control-Allow-Origin", "*")
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)
            return len(body)

        def do_GET(self):
            t0 = time.time()
            status, n = 500, 0
            try:
                m = _VHOST.match(self.path)
                if m:
                    op, vh = m.group(1), m.group(2)
                    ok = broker.create_vhost(vh) if op == "put" else broker.delete_vhost(vh)
                    status = 200 if ok is not None else 500   # any completed future -> 200 (A.Q27)
                    n = self._reply(status)
                elif self.path.rstrip("/") == "/admin/stats":
                    body = broker.stats_json()
                    if extra:
                        body = body[:-1] + "," + extra() + "}"
                    status, n = 200, self._reply(200, body.encode(), "application/json")
                elif self.path.rstrip("/") == "/admin/queues":
                    status, n = 200, self._reply(200, broker.queues_json().encode(), "application/json")
                elif self.path.rstrip("/") == "/admin/health":
                    status, n = 200, self._reply(200, b"ok")
                else:
                    status, n = 404, self._reply(404, b"not found")
            except Exception as e:  # noqa: BLE001 - report as 500 like the reference
                log.exception("admin request failed")
                status, n = 500, self._reply(500, str(e).encode())
            log.info("%s %s %d %.1fms %dB", self.command, self.path, status, (time.time() - t0) * 1000, n)

    return Handler


class AdminServer:
    def __init__(self, broker, port, host="127.0.0.1", extra=None):
        self.httpd = ThreadingHTTPServer((host, port), make_handler(broker, extra))
        self.port = self.httpd.server_address[1]
        self.thread = threading.Thread(target=self.httpd.serve_forever, name="chanamq-admin", daemon=True)

    def start(self):
        self.thread.start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()
