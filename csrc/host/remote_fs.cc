// WebHDFS and S3 over HTTP/1.1 (see remote_fs.h).
#include "remote_fs.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/hmac.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <pthread.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <map>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <utility>

#include "json.h"

namespace wh {
namespace host {

namespace {

std::string env(const char* k, const std::string& dflt = "") {
  const char* v = std::getenv(k);
  return v && *v ? std::string(v) : dflt;
}

std::string lower(std::string s) {
  for (auto& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}

// RFC 3986 unreserved characters pass; '/' too when keep_slash
std::string uri_encode(const std::string& s, bool keep_slash) {
  static const char* hex = "0123456789ABCDEF";
  std::string o;
  for (unsigned char c : s) {
    if (std::isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~' || (keep_slash && c == '/')) {
      o += (char)c;
    } else {
      o += '%';
      o += hex[c >> 4];
      o += hex[c & 15];
    }
  }
  return o;
}

std::string hexs(const unsigned char* p, size_t n) {
  static const char* hex = "0123456789abcdef";
  std::string o(2 * n, '0');
  for (size_t i = 0; i < n; ++i) o[2 * i] = hex[p[i] >> 4], o[2 * i + 1] = hex[p[i] & 15];
  return o;
}

std::string sha256_hex(const std::string& s) {
  unsigned char md[EVP_MAX_MD_SIZE];
  unsigned int n = 0;
  EVP_Digest(s.data(), s.size(), md, &n, EVP_sha256(), nullptr);
  return hexs(md, n);
}

std::string hmac(const std::string& key, const std::string& msg) {
  unsigned char md[EVP_MAX_MD_SIZE];
  unsigned int n = 0;
  HMAC(EVP_sha256(), key.data(), (int)key.size(),
       reinterpret_cast<const unsigned char*>(msg.data()), msg.size(), md, &n);
  return std::string(reinterpret_cast<char*>(md), n);
}

// ------------------------------------------------------------------ http
struct Url {
  bool tls = false;
  std::string host;
  int port = 80;
  std::string target = "/";  // path [?query]
  std::string hostport() const {
    return (tls ? port == 443 : port == 80) ? host : host + ":" + std::to_string(port);
  }
};

Url parse_url(const std::string& u) {
  Url r;
  size_t p;
  if (u.rfind("https://", 0) == 0) r.tls = true, r.port = 443, p = 8;
  else if (u.rfind("http://", 0) == 0) p = 7;
  else throw std::runtime_error("not an http(s) URL: " + u);
  const size_t slash = u.find('/', p);
  std::string hp = u.substr(p, slash == std::string::npos ? std::string::npos : slash - p);
  r.target = slash == std::string::npos ? "/" : u.substr(slash);
  if (!hp.empty() && hp[0] == '[') {  // [v6]:port
    const size_t e = hp.find(']');
    r.host = hp.substr(1, e - 1);
    if (e + 1 < hp.size() && hp[e + 1] == ':') r.port = std::atoi(hp.c_str() + e + 2);
  } else {
    const size_t c = hp.rfind(':');
    r.host = c == std::string::npos ? hp : hp.substr(0, c);
    if (c != std::string::npos) r.port = std::atoi(hp.c_str() + c + 1);
  }
  if (r.host.empty()) throw std::runtime_error("no host in URL " + u);
  return r;
}

// One client context per CA source: the system store, or the file named by
// SSL_CERT_FILE (OpenSSL's own variable, read when a context is made -- a
// context per value, so a process that changes it gets the new trust set).
// Peers are verified: chain and host name (or IP address).
SSL_CTX* tls_ctx() {
  static std::mutex mu;
  static std::map<std::string, SSL_CTX*> ctxs;
  const char* cf = std::getenv("SSL_CERT_FILE");
  const std::string key = cf ? cf : "";
  std::lock_guard<std::mutex> lk(mu);
  auto it = ctxs.find(key);
  if (it != ctxs.end()) return it->second;
  SSL_CTX* ctx = SSL_CTX_new(TLS_client_method());
  if (!ctx) throw std::runtime_error("TLS: cannot create a client context");
  SSL_CTX_set_default_verify_paths(ctx);
  SSL_CTX_set_verify(ctx, SSL_VERIFY_PEER, nullptr);
  ctxs[key] = ctx;
  return ctx;
}

bool is_ip_literal(const std::string& h) {
  unsigned char b[16];
  return inet_pton(AF_INET, h.c_str(), b) == 1 || inet_pton(AF_INET6, h.c_str(), b) == 1;
}

// SSL_write on a socket the peer closed raises SIGPIPE (OpenSSL's send has
// no MSG_NOSIGNAL): blocked on this thread for the write, and a pending one
// consumed, so a dropped connection is an error return, not a dead process
struct NoSigpipe {
  sigset_t old{}, pipe{};
  NoSigpipe() {
    sigemptyset(&pipe);
    sigaddset(&pipe, SIGPIPE);
    pthread_sigmask(SIG_BLOCK, &pipe, &old);
  }
  ~NoSigpipe() {
    sigset_t pend;
    sigpending(&pend);
    if (sigismember(&pend, SIGPIPE) && !sigismember(&old, SIGPIPE)) {
      timespec zero{0, 0};
      while (sigtimedwait(&pipe, nullptr, &zero) > 0) {
      }
    }
    pthread_sigmask(SIG_SETMASK, &old, nullptr);
  }
};

class Conn {
 public:
  explicit Conn(const Url& u) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_socktype = SOCK_STREAM;
    hints.ai_family = AF_UNSPEC;
    const std::string port = std::to_string(u.port);
    const int rc = getaddrinfo(u.host.c_str(), port.c_str(), &hints, &res);
    if (rc != 0) throw std::runtime_error("resolve " + u.host + ": " + gai_strerror(rc));
    for (addrinfo* a = res; a; a = a->ai_next) {
      fd_ = socket(a->ai_family, a->ai_socktype, a->ai_protocol);
      if (fd_ < 0) continue;
      timeval tv{60, 0};  // a stalled server ends the request, not the job
      setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
      setsockopt(fd_, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
      int one = 1;
      setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      if (connect(fd_, a->ai_addr, a->ai_addrlen) == 0) break;
      close(fd_);
      fd_ = -1;
    }
    freeaddrinfo(res);
    if (fd_ < 0) throw std::runtime_error("connect " + u.host + ":" + port + " failed");
    if (u.tls) {
      ssl_ = SSL_new(tls_ctx());
      SSL_set_fd(ssl_, fd_);
      if (is_ip_literal(u.host)) {  // an address: checked against the IP SANs, no SNI
        X509_VERIFY_PARAM_set1_ip_asc(SSL_get0_param(ssl_), u.host.c_str());
      } else {
        SSL_set_tlsext_host_name(ssl_, u.host.c_str());
        SSL_set1_host(ssl_, u.host.c_str());
      }
      NoSigpipe np;
      if (SSL_connect(ssl_) != 1) {
        char buf[256];
        ERR_error_string_n(ERR_get_error(), buf, sizeof buf);
        throw std::runtime_error("TLS handshake with " + u.host + ": " + buf);
      }
    }
  }
  Conn(const Conn&) = delete;
  Conn& operator=(const Conn&) = delete;
  ~Conn() {
    if (ssl_) SSL_free(ssl_);
    if (fd_ >= 0) close(fd_);
  }
  void write_all(const std::string& s) {
    NoSigpipe np;
    size_t off = 0;
    while (off < s.size()) {
      const int n = ssl_ ? SSL_write(ssl_, s.data() + off, (int)std::min<size_t>(s.size() - off, 1 << 20))
                         : (int)send(fd_, s.data() + off, s.size() - off, MSG_NOSIGNAL);
      if (n <= 0) throw std::runtime_error("http: send failed");
      off += (size_t)n;
    }
  }
  int read_some(char* buf, int n) {
    const int r = ssl_ ? SSL_read(ssl_, buf, n) : (int)recv(fd_, buf, n, 0);
    if (r < 0) throw std::runtime_error("http: receive failed (timeout or reset)");
    return r;
  }

 private:
  int fd_ = -1;
  SSL* ssl_ = nullptr;
};

struct Resp {
  int status = 0;
  std::map<std::string, std::string> hdr;  // lower-case names
  std::string body;
  std::string header(const std::string& k) const {
    auto it = hdr.find(k);
    return it == hdr.end() ? std::string() : it->second;
  }
};

using Headers = std::vector<std::pair<std::string, std::string>>;

// one request on a fresh connection (Connection: close: the response ends
// at EOF unless framed by Content-Length or chunked encoding)
Resp exchange(const std::string& method, const Url& u, const Headers& h, const std::string& body) {
  Conn c(u);
  std::string req = method + " " + u.target + " HTTP/1.1\r\nHost: " + u.hostport() +
                    "\r\nConnection: close\r\nUser-Agent: wormhole-amd\r\n";
  for (const auto& kv : h) req += kv.first + ": " + kv.second + "\r\n";
  if (!body.empty() || method == "PUT" || method == "POST")
    req += "Content-Length: " + std::to_string(body.size()) + "\r\n";
  req += "\r\n";
  c.write_all(req);
  if (!body.empty()) c.write_all(body);
  std::string raw;
  char buf[1 << 16];
  size_t hend = std::string::npos;
  int64_t clen = -1;
  bool chunked = false;
  Resp r;
  while (true) {
    const int n = c.read_some(buf, sizeof buf);
    if (n == 0) break;
    raw.append(buf, n);
    if (hend == std::string::npos) {
      hend = raw.find("\r\n\r\n");
      if (hend != std::string::npos) {
        // status line + headers
        size_t p = raw.find("\r\n");
        const std::string sl = raw.substr(0, p);
        const size_t sp = sl.find(' ');
        r.status = sp == std::string::npos ? 0 : std::atoi(sl.c_str() + sp + 1);
        while (p < hend) {
          const size_t q = raw.find("\r\n", p + 2);
          const std::string line = raw.substr(p + 2, q - p - 2);
          const size_t colon = line.find(':');
          if (colon != std::string::npos) {
            std::string v = line.substr(colon + 1);
            v.erase(0, v.find_first_not_of(" \t"));
            r.hdr[lower(line.substr(0, colon))] = v;
          }
          p = q;
        }
        if (r.hdr.count("content-length")) clen = std::atoll(r.hdr["content-length"].c_str());
        chunked = lower(r.header("transfer-encoding")).find("chunked") != std::string::npos;
        if (method == "HEAD" || r.status == 204 || r.status == 304) break;
      }
    }
    if (hend != std::string::npos && clen >= 0 && !chunked &&
        (int64_t)(raw.size() - hend - 4) >= clen)
      break;
  }
  if (hend == std::string::npos) throw std::runtime_error("http: no response header from " + u.host);
  std::string b = raw.substr(hend + 4);
  if (method == "HEAD") b.clear();
  if (chunked) {
    std::string out;
    size_t p = 0;
    while (p < b.size()) {
      const size_t e = b.find("\r\n", p);
      if (e == std::string::npos) break;
      const long n = std::strtol(b.substr(p, e - p).c_str(), nullptr, 16);
      if (n <= 0) break;
      out.append(b, e + 2, (size_t)n);
      p = e + 2 + (size_t)n + 2;
    }
    b.swap(out);
  } else if (clen >= 0 && (int64_t)b.size() > clen) {
    b.resize((size_t)clen);
  }
  r.body.swap(b);
  return r;
}

// follows redirects (the WebHDFS name node sends reads and writes on to a
// data node) and retries transient failures: connection errors and 5xx
Resp request(std::string method, std::string url, const Headers& h, const std::string& body,
             bool follow = true) {
  for (int attempt = 0;; ++attempt) {
    try {
      std::string m = method, u = url;
      for (int hop = 0; hop < 6; ++hop) {
        Resp r = exchange(m, parse_url(u), h, body);
        const bool redirect = r.status == 301 || r.status == 302 || r.status == 303 ||
                              r.status == 307 || r.status == 308;
        if (!(follow && redirect && !r.header("location").empty())) {
          if (r.status >= 500 && attempt < 3) throw std::runtime_error("http " + std::to_string(r.status));
          return r;
        }
        std::string loc = r.header("location");
        if (loc.rfind("http", 0) != 0) {  // relative
          const Url cur = parse_url(u);
          loc = std::string(cur.tls ? "https://" : "http://") + cur.hostport() + loc;
        }
        u = loc;
        if (r.status == 303) m = "GET";
      }
      throw std::runtime_error("http: too many redirects for " + url);
    } catch (const std::runtime_error& e) {
      if (attempt >= 3) throw;
      std::this_thread::sleep_for(std::chrono::milliseconds(200 << attempt));
    }
  }
}

[[noreturn]] void http_fail(const std::string& what, const std::string& uri, const Resp& r) {
  std::string b = r.body.substr(0, 300);
  throw std::runtime_error(what + " " + uri + ": HTTP " + std::to_string(r.status) + " " + b);
}

// ------------------------------------------------------------------ URIs
struct Parsed {
  std::string scheme, authority, path;  // path without the leading '/'
};

Parsed parse_uri(const std::string& uri) {
  const size_t sep = uri.find("://");
  if (sep == std::string::npos) throw std::runtime_error("not a URI: " + uri);
  Parsed p;
  p.scheme = lower(uri.substr(0, sep));
  std::string rest = uri.substr(sep + 3);
  const size_t slash = rest.find('/');
  p.authority = rest.substr(0, slash);
  p.path = slash == std::string::npos ? "" : rest.substr(slash + 1);
  return p;
}

bool is_s3(const std::string& s) { return s == "s3" || s == "s3a" || s == "s3n"; }
bool is_hdfs(const std::string& s) { return s == "hdfs" || s == "viewfs"; }

// ---------------------------------------------------------------- WebHDFS
std::string hdfs_url(const Parsed& p, const std::string& op) {
  std::string base = env("WH_WEBHDFS_URL");
  if (base.empty()) {
    std::string host = p.authority;
    const size_t c = host.rfind(':');
    if (c != std::string::npos && host.find(']') == std::string::npos) host = host.substr(0, c);
    if (host.empty()) throw std::runtime_error("hdfs URI without a name node: set WH_WEBHDFS_URL");
    base = "http://" + host + ":" + env("WH_WEBHDFS_PORT", "9870");
  }
  while (!base.empty() && base.back() == '/') base.pop_back();
  std::string u = base + "/webhdfs/v1/" + uri_encode(p.path, true) + "?op=" + op;
  const std::string user = env("HADOOP_USER_NAME", env("USER"));
  if (!user.empty()) u += "&user.name=" + uri_encode(user, false);
  return u;
}

// --------------------------------------------------------------------- S3
struct S3Target {
  Url ep;
  std::string bucket, key, region;
};

S3Target s3_of(const Parsed& p) {
  S3Target t;
  t.region = env("AWS_REGION", env("AWS_DEFAULT_REGION", "us-east-1"));
  t.ep = parse_url(env("WH_S3_ENDPOINT", "https://s3." + t.region + ".amazonaws.com"));
  t.bucket = p.authority;
  t.key = p.path;
  if (t.bucket.empty()) throw std::runtime_error("s3 URI without a bucket");
  return t;
}

std::string amz_now() {
  std::time_t now = std::time(nullptr);
  std::tm g;
  gmtime_r(&now, &g);
  char b[32];
  std::strftime(b, sizeof b, "%Y%m%dT%H%M%SZ", &g);
  return b;
}

// query: key -> value (unencoded); the canonical query sorts and encodes
Resp s3_request(const std::string& method, const S3Target& t, const std::string& key,
                const std::map<std::string, std::string>& query, Headers extra,
                const std::string& body) {
  std::string path = "/" + uri_encode(t.bucket, false);
  if (!key.empty()) path += "/" + uri_encode(key, true);
  std::string q;
  for (const auto& kv : query) {
    if (!q.empty()) q += "&";
    q += uri_encode(kv.first, false) + "=" + uri_encode(kv.second, false);
  }
  const std::string payload = sha256_hex(body);
  const std::string date = amz_now();
  const std::string id = env("AWS_ACCESS_KEY_ID"), secret = env("AWS_SECRET_ACCESS_KEY");
  const std::string token = env("AWS_SESSION_TOKEN");
  Headers h = std::move(extra);
  h.push_back({"x-amz-content-sha256", payload});
  h.push_back({"x-amz-date", date});
  if (!token.empty()) h.push_back({"x-amz-security-token", token});
  if (!id.empty() && !secret.empty())
    h.push_back({"Authorization", SigV4Authorization(method, t.ep.hostport(), path, q, date,
                                                     payload, t.region, id, secret, token)});
  std::string u = std::string(t.ep.tls ? "https://" : "http://") + t.ep.hostport() + path;
  if (!q.empty()) u += "?" + q;
  return request(method, u, h, body);
}

std::string xml_unescape(std::string s) {
  static const std::pair<const char*, const char*> m[] = {
      {"&lt;", "<"}, {"&gt;", ">"}, {"&quot;", "\""}, {"&apos;", "'"}, {"&amp;", "&"}};
  for (const auto& kv : m) {
    size_t p = 0;
    while ((p = s.find(kv.first, p)) != std::string::npos) {
      s.replace(p, std::strlen(kv.first), kv.second);
      p += std::strlen(kv.second);
    }
  }
  return s;
}

std::string xml_tag(const std::string& s, const std::string& tag, size_t from, size_t to,
                    size_t* at = nullptr) {
  const std::string o = "<" + tag + ">", c = "</" + tag + ">";
  const size_t a = s.find(o, from);
  if (a == std::string::npos || a >= to) return std::string();
  const size_t b = s.find(c, a);
  if (b == std::string::npos || b > to) return std::string();
  if (at) *at = b + c.size();
  return xml_unescape(s.substr(a + o.size(), b - a - o.size()));
}

}  // namespace

std::string SigV4Authorization(const std::string& method, const std::string& host,
                               const std::string& path, const std::string& query,
                               const std::string& amz_date, const std::string& payload_sha256,
                               const std::string& region, const std::string& key_id,
                               const std::string& secret, const std::string& token) {
  std::string ch = "host:" + host + "\nx-amz-content-sha256:" + payload_sha256 +
                   "\nx-amz-date:" + amz_date + "\n";
  std::string signed_h = "host;x-amz-content-sha256;x-amz-date";
  if (!token.empty()) {
    ch += "x-amz-security-token:" + token + "\n";
    signed_h += ";x-amz-security-token";
  }
  const std::string creq =
      method + "\n" + path + "\n" + query + "\n" + ch + "\n" + signed_h + "\n" + payload_sha256;
  const std::string day = amz_date.substr(0, 8);
  const std::string scope = day + "/" + region + "/s3/aws4_request";
  const std::string sts = "AWS4-HMAC-SHA256\n" + amz_date + "\n" + scope + "\n" + sha256_hex(creq);
  std::string k = hmac("AWS4" + secret, day);
  k = hmac(k, region);
  k = hmac(k, "s3");
  k = hmac(k, "aws4_request");
  const std::string sig = hmac(k, sts);
  return "AWS4-HMAC-SHA256 Credential=" + key_id + "/" + scope + ", SignedHeaders=" + signed_h +
         ", Signature=" + hexs(reinterpret_cast<const unsigned char*>(sig.data()), sig.size());
}

bool IsRemote(const std::string& uri) {
  const size_t sep = uri.find("://");
  if (sep == std::string::npos) return false;
  const std::string scheme = lower(uri.substr(0, sep));
  if (!is_s3(scheme) && !is_hdfs(scheme)) return false;
  std::string var = "WH_FS_MOUNT_";
  for (char c : scheme) var += (char)std::toupper((unsigned char)c);
  return env(var.c_str()).empty();  // a configured mount takes precedence
}

std::vector<RemoteEntry> RemoteList(const std::string& dir_uri) {
  const Parsed p = parse_uri(dir_uri);
  std::vector<RemoteEntry> out;
  std::string base = dir_uri;
  while (!base.empty() && base.back() == '/') base.pop_back();
  if (is_hdfs(p.scheme)) {
    Resp r = request("GET", hdfs_url(p, "LISTSTATUS"), {}, "");
    if (r.status == 404) return out;
    if (r.status != 200) http_fail("list", dir_uri, r);
    const Json j = Json::Parse(r.body);
    for (const Json& f : j["FileStatuses"]["FileStatus"].arr()) {
      if (f["type"].str() != "FILE") continue;
      const std::string sfx = f["pathSuffix"].str();
      out.push_back({sfx.empty() ? base : base + "/" + sfx, (int64_t)f["length"].num()});
    }
  } else {
    const S3Target t = s3_of(p);
    std::string prefix = t.key;
    if (!prefix.empty() && prefix.back() != '/') prefix += "/";
    const std::string root = p.scheme + "://" + t.bucket + "/";
    std::string token;
    do {
      std::map<std::string, std::string> q{{"list-type", "2"}, {"delimiter", "/"}};
      if (!prefix.empty()) q["prefix"] = prefix;
      if (!token.empty()) q["continuation-token"] = token;
      Resp r = s3_request("GET", t, "", q, {}, "");
      if (r.status != 200) http_fail("list", dir_uri, r);
      size_t at = 0;
      while (true) {
        const size_t a = r.body.find("<Contents>", at);
        if (a == std::string::npos) break;
        const size_t b = r.body.find("</Contents>", a);
        const std::string key = xml_tag(r.body, "Key", a, b);
        const std::string size = xml_tag(r.body, "Size", a, b);
        if (!key.empty() && key.back() != '/') out.push_back({root + key, std::atoll(size.c_str())});
        at = b;
      }
      token = xml_tag(r.body, "IsTruncated", 0, r.body.size()) == "true"
                  ? xml_tag(r.body, "NextContinuationToken", 0, r.body.size())
                  : std::string();
    } while (!token.empty());
    if (out.empty() && !t.key.empty()) {  // the URI names an object itself
      const int64_t n = RemoteSize(dir_uri);
      if (n >= 0) out.push_back({base, n});
    }
  }
  std::sort(out.begin(), out.end(),
            [](const RemoteEntry& a, const RemoteEntry& b) { return a.uri < b.uri; });
  return out;
}

int64_t RemoteSize(const std::string& uri) {
  const Parsed p = parse_uri(uri);
  if (is_hdfs(p.scheme)) {
    Resp r = request("GET", hdfs_url(p, "GETFILESTATUS"), {}, "");
    if (r.status == 404) return -1;
    if (r.status != 200) http_fail("stat", uri, r);
    const Json j = Json::Parse(r.body);
    return j["FileStatus"]["type"].str() == "FILE" ? (int64_t)j["FileStatus"]["length"].num() : -1;
  }
  const S3Target t = s3_of(p);
  Resp r = s3_request("HEAD", t, t.key, {}, {}, "");
  if (r.status == 404 || r.status == 403) return -1;
  if (r.status != 200) http_fail("stat", uri, r);
  return std::atoll(r.header("content-length").c_str());
}

std::string RemoteRead(const std::string& uri, int64_t off, int64_t len) {
  if (len <= 0) return std::string();
  const Parsed p = parse_uri(uri);
  if (is_hdfs(p.scheme)) {
    Resp r = request("GET", hdfs_url(p, "OPEN") + "&offset=" + std::to_string(off) +
                                "&length=" + std::to_string(len),
                     {}, "");
    if (r.status != 200) http_fail("read", uri, r);
    if ((int64_t)r.body.size() > len) r.body.resize((size_t)len);
    return r.body;
  }
  const S3Target t = s3_of(p);
  Resp r = s3_request("GET", t, t.key, {},
                      {{"Range", "bytes=" + std::to_string(off) + "-" + std::to_string(off + len - 1)}},
                      "");
  if (r.status == 416) return std::string();  // at / past the end
  if (r.status == 200) {  // (a server that ignores ranges: the whole object)
    return off < (int64_t)r.body.size() ? r.body.substr((size_t)off, (size_t)len) : std::string();
  }
  if (r.status != 206) http_fail("read", uri, r);
  return r.body;
}

void RemoteWrite(const std::string& uri, const std::string& data) {
  RemoteWriter w(uri);
  w.Write(data.data(), data.size());
  w.Close();
}

namespace {
// WebHDFS CREATE (PUT) / APPEND (POST): the name node answers 307 with the
// data node that takes the bytes
void hdfs_put(const std::string& uri, const std::string& op, const std::string& data) {
  const Parsed p = parse_uri(uri);
  const bool create = op == "CREATE";
  const std::string method = create ? "PUT" : "POST";
  Resp r = request(method, hdfs_url(p, op) + (create ? "&overwrite=true" : ""), {}, "", false);
  const std::string loc = r.header("location");
  if (r.status == 307 && !loc.empty())
    r = request(method, loc, {{"Content-Type", "application/octet-stream"}}, data);
  if (r.status != 201 && r.status != 200) http_fail(create ? "write" : "append", uri, r);
}
}  // namespace

RemoteWriter::RemoteWriter(const std::string& uri, int64_t part_bytes)
    : uri_(uri), part_(part_bytes > 0 ? part_bytes : (int64_t)64 << 20) {
  const Parsed p = parse_uri(uri);
  hdfs_ = is_hdfs(p.scheme);
  if (!hdfs_ && !is_s3(p.scheme)) throw std::runtime_error("not a remote URI: " + uri);
}

RemoteWriter::~RemoteWriter() {
  if (closed_ || hdfs_ || upload_id_.empty()) return;
  try {  // dropped unclosed: do not leave the parts billed in the bucket
    const S3Target t = s3_of(parse_uri(uri_));
    s3_request("DELETE", t, t.key, {{"uploadId", upload_id_}}, {}, "");
  } catch (...) {
  }
}

void RemoteWriter::Write(const char* p, size_t n) {
  if (closed_) throw std::runtime_error("write after close: " + uri_);
  buf_.append(p, n);
  while ((int64_t)buf_.size() >= part_) Part(false);
}

// uploads the first min(part, buffered) bytes (all of them when last)
void RemoteWriter::Part(bool last) {
  const size_t n = last ? buf_.size() : (size_t)std::min<int64_t>(part_, (int64_t)buf_.size());
  const std::string data = buf_.substr(0, n);
  if (hdfs_) {
    if (!created_) hdfs_put(uri_, "CREATE", data);
    else if (!data.empty()) hdfs_put(uri_, "APPEND", data);
    created_ = true;
  } else {
    const S3Target t = s3_of(parse_uri(uri_));
    if (upload_id_.empty()) {
      if (last) {  // the whole object fits one part: a plain PUT
        Resp r = s3_request("PUT", t, t.key, {}, {{"Content-Type", "application/octet-stream"}}, data);
        if (r.status != 200 && r.status != 201) http_fail("write", uri_, r);
        buf_.clear();
        ++nparts_;
        return;
      }
      Resp r = s3_request("POST", t, t.key, {{"uploads", ""}},
                          {{"Content-Type", "application/octet-stream"}}, "");
      if (r.status != 200) http_fail("create multipart upload", uri_, r);
      upload_id_ = xml_tag(r.body, "UploadId", 0, r.body.size());
      if (upload_id_.empty()) http_fail("create multipart upload (no UploadId)", uri_, r);
    }
    if (!data.empty() || etags_.empty()) {
      const std::string num = std::to_string(etags_.size() + 1);
      Resp r = s3_request("PUT", t, t.key, {{"partNumber", num}, {"uploadId", upload_id_}}, {}, data);
      if (r.status != 200) http_fail("upload part " + num, uri_, r);
      const std::string etag = r.header("etag");
      if (etag.empty()) http_fail("upload part " + num + " (no ETag)", uri_, r);
      etags_.push_back(etag);
    }
    if (last) {
      std::string x = "<CompleteMultipartUpload>";
      for (size_t i = 0; i < etags_.size(); ++i)
        x += "<Part><PartNumber>" + std::to_string(i + 1) + "</PartNumber><ETag>" + etags_[i] +
             "</ETag></Part>";
      x += "</CompleteMultipartUpload>";
      Resp r = s3_request("POST", t, t.key, {{"uploadId", upload_id_}},
                          {{"Content-Type", "application/xml"}}, x);
      // (S3 can answer 200 and still report an error in the body)
      if (r.status != 200 || r.body.find("<Error>") != std::string::npos)
        http_fail("complete multipart upload", uri_, r);
    }
  }
  ++nparts_;
  buf_.erase(0, n);
}

void RemoteWriter::Close() {
  if (closed_) return;
  Part(true);
  closed_ = true;
}

RemoteReader::RemoteReader(const std::string& uri, int64_t window) : uri_(uri), win_(window) {
  size_ = RemoteSize(uri);
  if (size_ < 0) throw std::runtime_error("cannot open " + uri);
}

RemoteReader::~RemoteReader() {
  if (next_.valid()) {
    try {
      next_.get();
    } catch (...) {
    }
  }
}

void RemoteReader::Fill() {
  if (pos_ >= buf_off_ && pos_ < buf_off_ + (int64_t)buf_.size()) return;
  // a read that continues the last window is sequential
  const bool seq = !buf_.empty() && pos_ == buf_off_ + (int64_t)buf_.size();
  if (next_.valid() && next_off_ == pos_) {
    buf_ = next_.get();  // (a failed read-ahead rethrows here)
    ++prefetched_;
  } else {
    if (next_.valid()) {  // the read-ahead was for another place: drop it
      try {
        next_.get();
      } catch (...) {
      }
    }
    buf_ = pos_ < size_ ? RemoteRead(uri_, pos_, std::min(win_, size_ - pos_)) : std::string();
  }
  buf_off_ = pos_;
  sequential_ = seq;
  const int64_t nx = buf_off_ + (int64_t)buf_.size();
  if (sequential_ && !buf_.empty() && nx < size_) {
    next_off_ = nx;
    const std::string uri = uri_;
    const int64_t len = std::min(win_, size_ - nx);
    next_ = std::async(std::launch::async, [uri, nx, len] { return RemoteRead(uri, nx, len); });
  }
}

size_t RemoteReader::Read(char* buf, size_t n) {
  size_t got = 0;
  while (got < n && pos_ < size_) {
    Fill();
    if (buf_.empty()) break;
    const int64_t in = (int64_t)buf_.size() - (pos_ - buf_off_);
    const size_t k = (size_t)std::min<int64_t>(in, (int64_t)(n - got));
    std::memcpy(buf + got, buf_.data() + (pos_ - buf_off_), k);
    got += k;
    pos_ += (int64_t)k;
  }
  return got;
}

int RemoteReader::GetC() {
  unsigned char c;
  return Read(reinterpret_cast<char*>(&c), 1) == 1 ? (int)c : -1;
}

}  // namespace host
}  // namespace wh
