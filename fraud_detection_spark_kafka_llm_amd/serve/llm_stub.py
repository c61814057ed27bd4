"""OpenAI-compatible stub LLM HTTP server (COMM-04 test double).

``POST /v1/chat/completions`` returns a deterministic completion (``llm.stub_completion``);
``GET /v1/models`` lists one model. Optional injected latency and failure modes (``fail_first``
HTTP 503s, then success) exercise the client's retry path. Runs in a daemon thread:

    with StubServer() as srv:
        client = ChatClient(base_url=srv.url)
"""
from __future__ import annotations

import json
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from .llm import stub_completion


class _Handler(BaseHTTPRequestHandler):
    server_version = "fdx-stub-llm/1.0"

    def log_message(self, *a):  # quiet
        pass

    def _send(self, code: int, body: dict) -> None:
        data = json.dumps(body).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def do_GET(self):  # noqa: N802
        if self.path.rstrip("/").endswith("/models"):
            self._send(200, {"object": "list", "data": [{"id": "stub-model", "object": "model"}]})
        else:
            self._send(404, {"error": "not found"})

    def do_POST(self):  # noqa: N802
        srv = self.server
        n = int(self.headers.get("Content-Length", "0"))
        try:
            body = json.loads(self.rfile.read(n) or b"{}")
        except ValueError:
            self._send(400, {"error": "bad json"})
            return
        if not self.path.rstrip("/").endswith("/chat/completions"):
            self._send(404, {"error": "not found"})
            return
        with srv.lock:
            srv.requests.append(body)
            fail = srv.fail_remaining > 0
            if fail:
                srv.fail_remaining -= 1
        if srv.latency_s:
            time.sleep(srv.latency_s)
        if fail:
            self._send(503, {"error": "injected failure"})
            return
        msgs = body.get("messages") or [{"content": ""}]
        text = stub_completion(msgs[-1].get("content", ""))
        self._send(200, {"id": "chatcmpl-stub", "object": "chat.completion", "model": body.get("model", "stub"),
                         "choices": [{"index": 0, "finish_reason": "stop",
                                      "message": {"role": "assistant", "content": text}}],
                         "usage": {"prompt_tokens": 0, "completion_tokens": 0, "total_tokens": 0}})


class StubServer:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, latency_s: float = 0.0, fail_first: int = 0):
        self.httpd = ThreadingHTTPServer((host, port), _Handler)
        self.httpd.lock = threading.Lock()
        self.httpd.requests = []
        self.httpd.latency_s = latency_s
        self.httpd.fail_remaining = fail_first
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True)

    @property
    def url(self) -> str:
        h, p = self.httpd.server_address[:2]
        return f"http://{h}:{p}/v1"

    @property
    def requests(self) -> list:
        return self.httpd.requests

    def start(self) -> "StubServer":
        self.thread.start()
        return self

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()


def main(argv=None) -> None:
    import argparse

    ap = argparse.ArgumentParser(description="OpenAI-compatible stub LLM server")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=1234)
    ap.add_argument("--latency", type=float, default=0.0)
    a = ap.parse_args(argv)
    srv = StubServer(a.host, a.port, a.latency)
    print(f"stub LLM listening on {srv.url}", flush=True)
    srv.httpd.serve_forever()


if __name__ == "__main__":
    main()
