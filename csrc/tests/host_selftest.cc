// Standalone self-test of the native host runtime (no torch, no GPU), built
// plain and under AddressSanitizer / ThreadSanitizer by
// `python build_native.py --sanitize address|thread` (the
// reference has no sanitizer targets; its host code had real races). It
// exercises every component that owns memory or threads: the LZ4 codec, the
// CRB row-block format, the text parsers, InputSplit part alignment (text
// and RecordIO), the multi-threaded ordered ThreadedReader / MinibatchIter,
// the conf parser, the WorkloadPool under concurrent workers and the
// control-plane transport (Van) with live reader threads.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "host/auc_host.h"
#include "host/common.h"
#include "host/io.h"
#include "host/json.h"
#include "host/parsers.h"
#include "host/van.h"
#include "host/workload_pool.h"

using namespace wh::host;

static int g_fail = 0;
#define EXPECT(c)                                                         \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);   \
      ++g_fail;                                                           \
    }                                                                     \
  } while (0)

static void test_lz4() {
  std::mt19937 rng(1);
  for (int kind = 0; kind < 3; ++kind) {
    for (int n : {0, 1, 7, 100, 4096, 300000}) {
      std::string src(n, '\0');
      for (int i = 0; i < n; ++i)
        src[i] = kind == 0 ? (char)rng() : kind == 1 ? (char)('a' + i % 7) : (char)(i / 1000);
      std::string dst(LZ4CompressBound(n) + 16, '\0');
      const int c = LZ4Compress(src.data(), &dst[0], n, (int)dst.size());
      EXPECT(c >= 0);
      std::string back(n + 8, '\0');
      const int d = LZ4Decompress(dst.data(), &back[0], c, n);
      EXPECT(d == n);
      EXPECT(std::memcmp(back.data(), src.data(), n) == 0);
    }
  }
  // malformed input must fail cleanly, never write out of bounds
  std::string junk(64, '\xff'), out(16, '\0');
  EXPECT(LZ4Decompress(junk.data(), &out[0], (int)junk.size(), (int)out.size()) < 0);
}

static RowBlock random_block(size_t rows, bool with_val, uint32_t seed) {
  std::mt19937_64 rng(seed);
  RowBlock b;
  for (size_t r = 0; r < rows; ++r) {
    b.label.push_back((float)(rng() % 2));
    const int len = 1 + (int)(rng() % 40);
    for (int j = 0; j < len; ++j) {
      b.index.push_back(rng());
      if (with_val) b.value.push_back((float)(rng() % 100) / 7.f);
    }
    b.offset.push_back((int64_t)b.index.size());
  }
  return b;
}

static bool same(const RowBlock& a, const RowBlock& b) {
  return a.label == b.label && a.offset == b.offset && a.index == b.index && a.value == b.value &&
         a.weight == b.weight;
}

static void test_crb() {
  for (bool v : {false, true}) {
    RowBlock b = random_block(1000, v, 7), d;
    const std::string enc = CRBEncode(b);
    CRBDecode(enc.data(), enc.size(), &d);
    EXPECT(same(b, d));
  }
}

static void test_parsers() {
  RowBlock b;
  const std::string svm = "1 3:0.5 9:1\n0 2:2\n\n1 7\n";
  ParseLibSVM(svm.data(), svm.data() + svm.size(), &b);
  EXPECT(b.size() == 3 && b.nnz() == 4);
  EXPECT(b.index[0] == 3 && b.index[3] == 7);
  const std::string crit = "1\t5\t\t3" + std::string(10, '\t') + "\tdeadbeef" +
                           std::string(25, '\t') + "\n";
  ParseCriteo(crit.data(), crit.data() + crit.size(), true, &b);
  EXPECT(b.size() == 1 && b.nnz() == 3);
  EXPECT((b.index[2] >> 54) == 13);  // first categorical field
  const std::string adfea = "1 2 1 5:3 9:4\n";
  ParseAdfea(adfea.data(), adfea.data() + adfea.size(), &b);
  EXPECT(b.size() == 1 && b.nnz() == 2);
}

static std::string tmpfile(const char* name) {
  const char* d = std::getenv("TMPDIR");
  return std::string(d && *d ? d : "/tmp") + "/wh_selftest_" + name;
}

static void test_splits_and_reader() {
  // text: every line lands in exactly one of n parts, in order
  const std::string path = tmpfile("text.svm");
  {
    std::FILE* f = std::fopen(path.c_str(), "wb");
    for (int i = 0; i < 20000; ++i) std::fprintf(f, "%d %d:1 %d:2\n", i % 2, i, i + 1);
    std::fclose(f);
  }
  for (int n : {1, 3, 16}) {
    std::vector<uint64_t> seen;
    for (int k = 0; k < n; ++k) {
      BlockReader r(path, k, n, "libsvm");
      RowBlock b;
      while (r.Next(&b))
        for (size_t i = 0; i < b.size(); ++i) seen.push_back(b.index[b.offset[i]]);
    }
    EXPECT(seen.size() == 20000);
    for (size_t i = 0; i < seen.size(); ++i) EXPECT(seen[i] == i);
  }
  // RecordIO (CRB): parts align to records, every record once
  const std::string crb = tmpfile("blocks.crb");
  std::vector<RowBlock> blocks;
  {
    RecordIOWriter w(crb);
    for (int i = 0; i < 50; ++i) {
      blocks.push_back(random_block(100 + i, i % 2 == 0, 100 + i));
      w.WriteRecord(CRBEncode(blocks.back()));
    }
    w.Close();
  }
  for (int n : {1, 4, 13}) {
    size_t got = 0;
    for (int k = 0; k < n; ++k) {
      BlockReader r(crb, k, n, "crb");
      RowBlock b;
      while (r.Next(&b)) {
        EXPECT(got < blocks.size() && same(b, blocks[got]));
        ++got;
      }
    }
    EXPECT(got == blocks.size());
  }
  // many parser threads hand out chunks in read order
  std::vector<std::vector<uint64_t>> runs;
  for (int nt : {1, 8}) {
    ThreadedReader tr(path, 0, 1, "libsvm", nt);
    RowBlock b;
    std::vector<uint64_t> ids;
    while (tr.Next(&b)) ids.insert(ids.end(), b.index.begin(), b.index.end());
    runs.push_back(ids);
  }
  EXPECT(runs[0] == runs[1] && runs[0].size() == 40000);
  // early destruction with workers still running must not leak or race
  for (int i = 0; i < 5; ++i) {
    ThreadedReader tr(path, 0, 1, "libsvm", 8);
    RowBlock b;
    tr.Next(&b);
  }
  // minibatches with the shuffle buffer and negative sampling
  MinibatchIter it(path, 0, 1, "libsvm", 1000, 5000, 0.5f, 3, 4);
  size_t rows = 0;
  while (it.Next()) rows += it.Value().size();
  EXPECT(rows > 12000 && rows < 18000);  // all positives + about half the negatives
  std::remove(path.c_str());
  std::remove(crb.c_str());
}

static void test_conf() {
  auto items = ParseConf("# c\nminibatch = 1000\nembedding {\n dim = 16\n}\nname: \"x y\"\n");
  EXPECT(items.size() == 3);
  EXPECT(items[0].key == "minibatch" && items[0].value == "1000");
  EXPECT(items[1].kind == 'm' && items[1].children.size() == 1);
  EXPECT(items[2].kind == 's' && items[2].value == "x y");
}

static void test_pool_concurrent() {
  WorkloadPool pool(true, 5, 2.0, 5.0, 10, 0.05);
  std::vector<std::string> files;
  for (int i = 0; i < 20; ++i) files.push_back("f" + std::to_string(i));
  pool.Add(files, 10);
  std::atomic<int> done{0};
  std::vector<std::thread> th;
  for (int w = 0; w < 8; ++w) {
    th.emplace_back([&, w] {
      const std::string me = "worker-" + std::to_string(w);
      Assignment a;
      int resets = 0;
      while (pool.Get(me, &a)) {
        if (w == 3 && resets < 3) {
          ++resets;
          pool.Reset(me);  // a failure: the part goes back to the pool
          continue;
        }
        pool.FinishOne(me, a.filename, a.k);
        done.fetch_add(1);
      }
    });
  }
  for (auto& t : th) t.join();
  EXPECT(pool.IsFinished());
  EXPECT(pool.num_finished() == 200);
}

static void test_json() {
  // the control-plane messages: Python json.dumps output in, ours out
  Json d = Json::Parse(
      "{\"msg\": \"request\", \"finished\": {\"file\": \"a\\\"b\\u00e9\", \"k\": 3},"
      " \"data\": [1.5, -2e-3, 0, NaN], \"files\": [], \"x\": null, \"ok\": true}");
  EXPECT(d["msg"].str() == "request");
  EXPECT(d["finished"]["k"].num() == 3);
  EXPECT(d["finished"]["file"].str() == "a\"b\xc3\xa9");
  const auto v = d["data"].nums();
  EXPECT(v.size() == 4 && v[0] == 1.5 && v[1] == -2e-3 && v[3] != v[3]);
  EXPECT(d["files"].strs().empty() && d["x"].is_null() && d["ok"].truthy());
  EXPECT(!d["missing"].truthy());
  Json o = Json::Obj().set("cmd", Json::Str("workload")).set("file", Json::Null())
               .set("k", Json::Num(7)).set("w", Json::Num(0.25));
  Json back = Json::Parse(o.Dump());
  EXPECT(back["cmd"].str() == "workload" && back["file"].is_null());
  EXPECT(back["k"].num() == 7 && back["w"].num() == 0.25);
  bool threw = false;
  try {
    Json::Parse("{\"a\": }");
  } catch (const std::exception&) {
    threw = true;
  }
  EXPECT(threw);
}

static void test_van() {
  // control-plane transport: 4 clients x 200 frames into one listener, and
  // replies back, with every connection's reader thread live
  Van server;
  const int port = server.Listen(0);
  EXPECT(port > 0);
  std::vector<std::thread> th;
  std::atomic<int> replies{0};
  for (int c = 0; c < 4; ++c) {
    th.emplace_back([&, c] {
      Van cl;
      const std::string me = "client-" + std::to_string(c);
      cl.Connect("127.0.0.1", port, me, 10.0);
      for (int i = 0; i < 200; ++i) EXPECT(cl.Send("scheduler", me + ":" + std::to_string(i)));
      std::string from, msg;
      int got = 0;
      while (got < 200 && cl.Recv(10.0, &from, &msg)) ++got;
      replies.fetch_add(got);
      cl.Close();
    });
  }
  int n = 0;
  std::string from, msg;
  while (n < 800 && server.Recv(10.0, &from, &msg)) {
    if (msg == "__closed__") continue;  // a client that already got all its acks
    ++n;
    EXPECT(msg.rfind(from + ":", 0) == 0);
    EXPECT(server.Send(from, "ack"));
  }
  EXPECT(n == 800);
  for (auto& t : th) t.join();
  EXPECT(replies.load() == 800);
  server.Close();
}

// the host AUC against an O(n^2) count of the same definition (key order:
// score bits, then index)
static void test_auc() {
  std::mt19937 rng(5);
  std::vector<uint64_t> ws;
  for (int n : {1, 2, 3, 17, 400, 3000}) {
    for (int kind = 0; kind < 3; ++kind) {
      std::vector<float> p(n), l(n);
      for (int i = 0; i < n; ++i) {
        p[i] = kind == 0 ? (float)(rng() % 1000) / 999.f
                         : kind == 1 ? (float)(rng() % 4) * (rng() % 2 ? -1.f : 1.f) : 0.5f;
        l[i] = (rng() % 3) == 0 ? 1.f : 0.f;
      }
      uint64_t tot = 0, tp = 0;
      for (int i = 0; i < n; ++i) tp += l[i] > 0.f;
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
          if (!(l[i] > 0.f) || l[j] > 0.f) continue;
          const uint32_t a = wh::auc_ord_bits(p[i]), b = wh::auc_ord_bits(p[j]);
          tot += a < b || (a == b && i < j);
        }
      double want = 1.0;
      if (tp != 0 && tp != (uint64_t)n) {
        const double r = (double)tot / ((double)tp * (double)(n - tp));
        want = r < 0.5 ? 1 - r : r;
      }
      EXPECT(wh::auc_exact_host(p.data(), l.data(), n, ws) == want);
    }
  }
}

int main() {
  test_auc();
  test_lz4();
  test_crb();
  test_parsers();
  test_splits_and_reader();
  test_conf();
  test_pool_concurrent();
  test_json();
  test_van();
  if (g_fail) {
    std::fprintf(stderr, "host_selftest: %d failure(s)\n", g_fail);
    return 1;
  }
  std::printf("host_selftest: ok\n");
  return 0;
}
