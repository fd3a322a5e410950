"""A local stand-in for an HDFS name node + data node (WebHDFS REST) and an
S3 endpoint (ListObjectsV2, HEAD, ranged GET, PUT, with AWS Signature V4
checked by an implementation of its own), serving a directory tree -- what
the native remote file systems (csrc/host/remote_fs.cc) are tested against.

    srv = MockRemote(root, access_key="AK", secret_key="SK"); srv.start()
    ... WH_WEBHDFS_PORT=srv.port, WH_S3_ENDPOINT=srv.url ...
    srv.stop()

With certfile / keyfile the endpoint is HTTPS (tests point SSL_CERT_FILE at
the certificate). WebHDFS: /webhdfs/v1/<path>?op=LISTSTATUS|GETFILESTATUS|OPEN|CREATE|APPEND
(OPEN, CREATE and APPEND answer 307 to /datanode/<path>, like a name node).
S3: path-style /<bucket>/<key> under <root>/<bucket>; listings paginate 2 keys
at a time; multipart uploads (create, upload part with ETags, complete with
the part list checked, abort).
"""
import hashlib
import hmac
import json
import os
import re
import ssl
import threading
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer


def sigv4(method, host, path, query, amz_date, payload, region, key_id, secret, token=""):
    """AWS Signature V4 for S3 (an independent Python version of the one in
    csrc/host/remote_fs.cc)."""
    ch = "host:%s\nx-amz-content-sha256:%s\nx-amz-date:%s\n" % (host, payload, amz_date)
    sh = "host;x-amz-content-sha256;x-amz-date"
    if token:
        ch += "x-amz-security-token:%s\n" % token
        sh += ";x-amz-security-token"
    creq = "\n".join([method, path, query, ch, sh, payload])
    day = amz_date[:8]
    scope = "%s/%s/s3/aws4_request" % (day, region)
    sts = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope,
                     hashlib.sha256(creq.encode()).hexdigest()])

    def h(k, m):
        return hmac.new(k, m.encode(), hashlib.sha256).digest()
    k = h(h(h(h(("AWS4" + secret).encode(), day), region), "s3"), "aws4_request")
    sig = hmac.new(k, sts.encode(), hashlib.sha256).hexdigest()
    return "AWS4-HMAC-SHA256 Credential=%s/%s, SignedHeaders=%s, Signature=%s" % (
        key_id, scope, sh, sig)


def _enc(s, safe):
    return urllib.parse.quote(s, safe=safe)


class _Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"

    def log_message(self, *a):  # quiet
        pass

    # ------------------------------------------------------------ helpers
    def _send(self, code, body=b"", headers=None):
        self.send_response(code)
        for k, v in (headers or {}).items():
            self.send_header(k, v)
        self.send_header("Content-Length", str(len(body)))
        self.send_header("Connection", "close")
        self.end_headers()
        if self.command != "HEAD":
            self.wfile.write(body)
        self.server.log.append((self.command, self.path, code))

    def _body(self):
        n = int(self.headers.get("Content-Length") or 0)
        return self.rfile.read(n) if n else b""

    def _local(self, rel):
        p = os.path.normpath(os.path.join(self.server.root, rel.lstrip("/")))
        assert p.startswith(self.server.root)
        return p

    # ----------------------------------------------------------- dispatch
    def _route(self):
        u = urllib.parse.urlsplit(self.path)
        q = dict(urllib.parse.parse_qsl(u.query, keep_blank_values=True))
        path = urllib.parse.unquote(u.path)
        if path.startswith("/webhdfs/v1/"):
            return self._webhdfs(path[len("/webhdfs/v1"):], q)
        if path.startswith("/datanode/"):
            return self._datanode(path[len("/datanode"):], q)
        return self._s3(u, path, q)

    do_GET = do_PUT = do_HEAD = do_POST = do_DELETE = lambda self: self._route()

    # ------------------------------------------------------------ WebHDFS
    def _webhdfs(self, path, q):
        if self.server.hdfs_user and q.get("user.name") != self.server.hdfs_user:
            return self._send(403, b'{"RemoteException":{"message":"bad user"}}')
        op = q.get("op")
        local = self._local(path)
        if op == "GETFILESTATUS":
            if not os.path.exists(local):
                return self._send(404, b'{"RemoteException":{"message":"not found"}}')
            st = {"type": "DIRECTORY" if os.path.isdir(local) else "FILE",
                  "length": 0 if os.path.isdir(local) else os.path.getsize(local)}
            return self._send(200, json.dumps({"FileStatus": st}).encode())
        if op == "LISTSTATUS":
            if not os.path.exists(local):
                return self._send(404, b'{"RemoteException":{"message":"not found"}}')
            if os.path.isfile(local):
                ent = [{"pathSuffix": "", "type": "FILE", "length": os.path.getsize(local)}]
            else:
                ent = []
                for n in sorted(os.listdir(local)):
                    f = os.path.join(local, n)
                    ent.append({"pathSuffix": n, "type": "DIRECTORY" if os.path.isdir(f) else "FILE",
                                "length": 0 if os.path.isdir(f) else os.path.getsize(f)})
            return self._send(200, json.dumps({"FileStatuses": {"FileStatus": ent}}).encode())
        if op in ("OPEN", "CREATE", "APPEND"):
            loc = "%s/datanode%s?%s" % (self.server.base_url, _enc(path, "/"),
                                        urllib.parse.urlencode(q))
            return self._send(307, b"", {"Location": loc})
        return self._send(400, b"unsupported op")

    def _datanode(self, path, q):
        local = self._local(path)
        if self.command == "POST" and q.get("op") == "APPEND":
            if not os.path.isfile(local):
                return self._send(404)
            with open(local, "ab") as f:
                f.write(self._body())
            return self._send(200)
        if self.command == "PUT":
            os.makedirs(os.path.dirname(local), exist_ok=True)
            with open(local, "wb") as f:
                f.write(self._body())
            return self._send(201)
        if not os.path.isfile(local):
            return self._send(404)
        data = open(local, "rb").read()
        off = int(q.get("offset", 0))
        n = int(q.get("length", len(data)))
        return self._send(200, data[off:off + n])

    # ----------------------------------------------------------------- S3
    def _s3_auth_ok(self, u, path):
        if not self.server.secret_key:
            return True
        auth = self.headers.get("Authorization", "")
        pairs = sorted(urllib.parse.parse_qsl(u.query, keep_blank_values=True))
        cq = "&".join("%s=%s" % (_enc(k, "-_.~"), _enc(v, "-_.~")) for k, v in pairs)
        want = sigv4(self.command, self.headers["Host"], _enc(path, "/-_.~"), cq,
                     self.headers.get("x-amz-date", ""),
                     self.headers.get("x-amz-content-sha256", ""), self.server.region,
                     self.server.access_key, self.server.secret_key)
        body_ok = True
        if self.command in ("PUT", "POST"):
            body_ok = hashlib.sha256(self._peek_body()).hexdigest() == \
                self.headers.get("x-amz-content-sha256")
        return hmac.compare_digest(auth, want) and body_ok

    def _peek_body(self):
        if not hasattr(self, "_bodybuf"):
            self._bodybuf = self._body()
        return self._bodybuf

    def _s3(self, u, path, q):
        if not self._s3_auth_ok(u, path):
            self.server.denied += 1
            return self._send(403, b"<Error><Code>SignatureDoesNotMatch</Code></Error>")
        parts = path.lstrip("/").split("/", 1)
        bucket, key = parts[0], parts[1] if len(parts) > 1 else ""
        broot = os.path.join(self.server.root, bucket)
        if not key and self.command == "GET" and q.get("list-type") == "2":
            prefix = q.get("prefix", "")
            keys = []
            for dp, _, fns in os.walk(broot):
                for fn in fns:
                    k = os.path.relpath(os.path.join(dp, fn), broot).replace(os.sep, "/")
                    if k.startswith(prefix) and "/" not in k[len(prefix):]:
                        keys.append(k)
            keys.sort()
            start = q.get("continuation-token")
            if start:
                keys = [k for k in keys if k > start]
            page, more = keys[:2], len(keys) > 2
            xml = "<ListBucketResult>" + "".join(
                "<Contents><Key>%s</Key><Size>%d</Size></Contents>" % (
                    k.replace("&", "&amp;"), os.path.getsize(os.path.join(broot, k)))
                for k in page)
            xml += "<IsTruncated>%s</IsTruncated>" % ("true" if more else "false")
            if more:
                xml += "<NextContinuationToken>%s</NextContinuationToken>" % page[-1]
            xml += "</ListBucketResult>"
            return self._send(200, xml.encode(), {"Content-Type": "application/xml"})
        local = os.path.join(broot, key)
        ups = self.server.uploads
        if self.command == "POST" and "uploads" in q:  # CreateMultipartUpload
            uid = "up%d" % len(self.server.upload_ids)
            self.server.upload_ids.append(uid)
            ups[uid] = (key, {})
            return self._send(200, ("<InitiateMultipartUploadResult><UploadId>%s</UploadId>"
                                    "</InitiateMultipartUploadResult>" % uid).encode())
        if "uploadId" in q:
            uid = q["uploadId"]
            if uid not in ups or ups[uid][0] != key:
                return self._send(404, b"<Error><Code>NoSuchUpload</Code></Error>")
            parts = ups[uid][1]
            if self.command == "PUT":  # UploadPart
                data = self._peek_body()
                etag = '"%s"' % hashlib.md5(data).hexdigest()
                parts[int(q["partNumber"])] = (etag, data)
                return self._send(200, b"", {"ETag": etag})
            if self.command == "DELETE":  # AbortMultipartUpload
                del ups[uid]
                self.server.aborted += 1
                return self._send(204)
            if self.command == "POST":  # CompleteMultipartUpload
                body = self._peek_body().decode()
                listed = re.findall(r"<Part><PartNumber>(\d+)</PartNumber><ETag>(.*?)</ETag></Part>", body)
                nums = [int(n) for n, _ in listed]
                if not listed or nums != sorted(nums) or any(parts.get(int(n), ("",))[0] != e
                                                             for n, e in listed):
                    return self._send(400, b"<Error><Code>InvalidPart</Code></Error>")
                os.makedirs(os.path.dirname(local), exist_ok=True)
                with open(local, "wb") as f:
                    for n, _ in listed:
                        f.write(parts[int(n)][1])
                del ups[uid]
                return self._send(200, b"<CompleteMultipartUploadResult></CompleteMultipartUploadResult>")
        if self.command == "PUT":
            os.makedirs(os.path.dirname(local), exist_ok=True)
            with open(local, "wb") as f:
                f.write(self._peek_body())
            return self._send(200)
        if not os.path.isfile(local):
            return self._send(404, b"<Error><Code>NoSuchKey</Code></Error>")
        data = open(local, "rb").read()
        if self.command == "HEAD":
            self.send_response(200)
            self.send_header("Content-Length", str(len(data)))
            self.send_header("Connection", "close")
            self.end_headers()
            self.server.log.append(("HEAD", self.path, 200))
            return None
        rng = self.headers.get("Range")
        if rng:
            a, b = rng.split("=", 1)[1].split("-")
            a, b = int(a), min(int(b), len(data) - 1)
            if a >= len(data):
                return self._send(416)
            return self._send(206, data[a:b + 1])
        return self._send(200, data)


class MockRemote:
    """certfile / keyfile: serve HTTPS (the URLs then name `host`, which the
    certificate must carry)."""

    def __init__(self, root, access_key="", secret_key="", region="us-east-1", hdfs_user="",
                 certfile=None, keyfile=None, host="127.0.0.1"):
        self.httpd = ThreadingHTTPServer(("127.0.0.1", 0), _Handler)
        if certfile:
            ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
            ctx.load_cert_chain(certfile, keyfile)
            self.httpd.socket = ctx.wrap_socket(self.httpd.socket, server_side=True)
        self.httpd.daemon_threads = True
        self.httpd.root = os.path.abspath(root)
        self.httpd.access_key, self.httpd.secret_key = access_key, secret_key
        self.httpd.region = region
        self.httpd.hdfs_user = hdfs_user
        self.httpd.log = []
        self.httpd.denied = 0
        self.httpd.uploads, self.httpd.upload_ids, self.httpd.aborted = {}, [], 0
        self.port = self.httpd.server_address[1]
        self.url = "%s://%s:%d" % ("https" if certfile else "http", host, self.port)
        self.httpd.base_url = self.url
        self.th = threading.Thread(target=self.httpd.serve_forever, daemon=True)

    @property
    def log(self):
        return self.httpd.log

    @property
    def denied(self):
        return self.httpd.denied

    @property
    def aborted(self):
        return self.httpd.aborted

    @property
    def open_uploads(self):
        return len(self.httpd.uploads)

    def start(self):
        self.th.start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()

    def env(self, creds=True):
        """The environment a client of this server needs."""
        e = {"WH_WEBHDFS_PORT": str(self.port), "WH_S3_ENDPOINT": self.url,
             "AWS_REGION": self.httpd.region}
        if self.url.startswith("https"):
            e["WH_WEBHDFS_URL"] = self.url
        if creds and self.httpd.secret_key:
            e.update(AWS_ACCESS_KEY_ID=self.httpd.access_key,
                     AWS_SECRET_ACCESS_KEY=self.httpd.secret_key)
        if self.httpd.hdfs_user:
            e["HADOOP_USER_NAME"] = self.httpd.hdfs_user
        return e
