// Native HiveServer2 (TCLIService, Thrift binary protocol) front end.
//
// The reference fronts its cluster with Spark's HiveThriftServer2 (a JVM server, one thread per
// JDBC connection: asql/hive/thriftserver/sparklinedata/HiveThriftServer2.scala:55-79) and drives
// it with many concurrent BI clients (docs/bi-benchmark/snap-sales-demo.jmx:87-101).  A pure-Python
// server is GIL-bound long before the GPU is busy (profiles/: 1.1 cores, ~1.4 ms of interpreter time
// per statement, the GPU ~11% busy at 800 QPS).  This gateway moves everything that scales with the
// number of *statements* out of the interpreter:
//
//   * one native thread per connection: SASL PLAIN handshake, framed / unframed message I/O,
//     Thrift binary decoding and encoding;
//   * ExecuteStatement of a query (SELECT / WITH / '(') is keyed by (session context token, text);
//     identical statements that are still waiting join the pending batch (one execution for all of
//     them -- never a result computed before the request arrived);
//   * GetOperationStatus, GetResultSetMetadata, FetchResults (column-based TRowSet pages sliced
//     from the batch's typed columns), CloseOperation and CancelOperation of those operations.
//
// Python keeps what scales with *executions*: executor threads pull batches (next_batch releases the
// GIL while waiting), run the statement on the leader's session and hand back typed columns once.
// Every other RPC (OpenSession, commands such as SET / USE / CREATE, metadata calls, statements with
// a confOverlay or timeout) is forwarded as raw message bytes to the Python server, which also
// publishes each session's context token (conf + current database + temp views) after it changes.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

// ------------------------------------------------------------------ thrift wire constants
enum : int8_t { T_STOP = 0, T_BOOL = 2, T_BYTE = 3, T_DOUBLE = 4, T_I16 = 6, T_I32 = 8, T_I64 = 10,
                T_STRING = 11, T_STRUCT = 12, T_MAP = 13, T_SET = 14, T_LIST = 15 };
constexpr uint32_t VERSION_1 = 0x80010000u;
constexpr int REPLY = 2;
enum : int32_t { OP_INITIALIZED = 0, OP_RUNNING = 1, OP_FINISHED = 2, OP_CANCELED = 3, OP_ERROR = 5 };
constexpr int SASL_START = 1, SASL_BAD = 3, SASL_COMPLETE = 5;

struct ProtocolError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::system_clock::now().time_since_epoch()).count();
}

double steady_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ------------------------------------------------------------------ writer (big endian)
struct W {
  std::string b;
  void i8(int8_t v) { b.push_back(static_cast<char>(v)); }
  void i16(int16_t v) { uint16_t u = htons(static_cast<uint16_t>(v)); b.append(reinterpret_cast<char*>(&u), 2); }
  void i32(int32_t v) { uint32_t u = htonl(static_cast<uint32_t>(v)); b.append(reinterpret_cast<char*>(&u), 4); }
  void i64(int64_t v) {
    uint64_t u = static_cast<uint64_t>(v);
    char t[8];
    for (int i = 0; i < 8; ++i) t[i] = static_cast<char>((u >> (56 - 8 * i)) & 0xff);
    b.append(t, 8);
  }
  void dbl(double v) { int64_t x; std::memcpy(&x, &v, 8); i64(x); }
  void str(const std::string& s) { i32(static_cast<int32_t>(s.size())); b += s; }
  void str(const char* p, size_t n) { i32(static_cast<int32_t>(n)); b.append(p, n); }
  void field(int8_t t, int16_t id) { i8(t); i16(id); }
  void stop() { i8(T_STOP); }
  void msg(const std::string& name, int32_t seqid) {
    i32(static_cast<int32_t>(VERSION_1 | REPLY));
    str(name);
    i32(seqid);
  }
};

// ------------------------------------------------------------------ reader + generic value tree
struct R {
  const uint8_t* p;
  size_t n, o = 0;
  R(const std::string& s) : p(reinterpret_cast<const uint8_t*>(s.data())), n(s.size()) {}
  void need(size_t k) { if (o + k > n) throw ProtocolError("truncated message"); }
  int8_t i8() { need(1); return static_cast<int8_t>(p[o++]); }
  int16_t i16() { need(2); int16_t v = static_cast<int16_t>((p[o] << 8) | p[o + 1]); o += 2; return v; }
  int32_t i32() {
    need(4);
    uint32_t v = (uint32_t(p[o]) << 24) | (uint32_t(p[o + 1]) << 16) | (uint32_t(p[o + 2]) << 8) | p[o + 3];
    o += 4;
    return static_cast<int32_t>(v);
  }
  int64_t i64() {
    need(8);
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | p[o + i];
    o += 8;
    return static_cast<int64_t>(v);
  }
  std::string str() {
    int32_t k = i32();
    if (k < 0) throw ProtocolError("negative length");
    need(static_cast<size_t>(k));
    std::string s(reinterpret_cast<const char*>(p + o), static_cast<size_t>(k));
    o += static_cast<size_t>(k);
    return s;
  }
};

struct Node {  // one decoded thrift value (only what the native RPCs read)
  int8_t t = T_STOP;
  int64_t i = 0;
  double d = 0;
  std::string s;
  std::unordered_map<int16_t, std::unique_ptr<Node>> f;  // struct fields
  size_t nlist = 0;                                      // list / set / map length (elements skipped)
  const Node* get(int16_t id) const { auto it = f.find(id); return it == f.end() ? nullptr : it->second.get(); }
};

void read_value(R& r, int8_t t, Node& out, int depth = 0) {
  if (depth > 64) throw ProtocolError("nesting too deep");
  out.t = t;
  switch (t) {
    case T_BOOL: case T_BYTE: out.i = r.i8(); break;
    case T_I16: out.i = r.i16(); break;
    case T_I32: out.i = r.i32(); break;
    case T_I64: out.i = r.i64(); break;
    case T_DOUBLE: { int64_t x = r.i64(); std::memcpy(&out.d, &x, 8); break; }
    case T_STRING: out.s = r.str(); break;
    case T_STRUCT:
      for (;;) {
        int8_t ft = r.i8();
        if (ft == T_STOP) break;
        int16_t id = r.i16();
        auto& slot = out.f[id];
        slot.reset(new Node());
        read_value(r, ft, *slot, depth + 1);
      }
      break;
    case T_MAP: {
      int8_t kt = r.i8(), vt = r.i8();
      int32_t k = r.i32();
      if (k < 0) throw ProtocolError("negative map size");
      out.nlist = static_cast<size_t>(k);
      for (int32_t j = 0; j < k; ++j) {
        Node kn, vn;
        read_value(r, kt, kn, depth + 1);
        read_value(r, vt, vn, depth + 1);
      }
      break;
    }
    case T_LIST: case T_SET: {
      int8_t et = r.i8();
      int32_t k = r.i32();
      if (k < 0) throw ProtocolError("negative list size");
      out.nlist = static_cast<size_t>(k);
      for (int32_t j = 0; j < k; ++j) {
        Node tmp;
        read_value(r, et, tmp, depth + 1);
      }
      break;
    }
    default: throw ProtocolError("unknown thrift type");
  }
}

// ------------------------------------------------------------------ batches, operations
struct Col {
  int kind = 6;            // 0 bool 1 byte 2 i16 3 i32 4 i64 5 double 6 string
  std::string data;        // fixed-width little-endian values, or the utf-8 blob
  std::vector<int64_t> off;  // strings: n + 1 offsets into data
  std::string nulls;       // one byte per row, 1 = NULL
};

struct Batch {
  int64_t id = 0;
  std::string sid, stmt, key;
  int state = OP_INITIALIZED;
  std::string error, schema;  // schema: an encoded TTableSchema struct (from Python)
  std::vector<Col> cols;
  int64_t nrows = 0, started = 0, completed = 0;
  double queued_at = 0.0;  // steady-clock seconds at enqueue (admission wait = pick-up - this)
  int live = 0, cancels = 0;
  bool cancel = false;
};

struct Op {
  std::shared_ptr<Batch> b;
  std::string secret, sid;
  int64_t cursor = 0;
  bool cancelled = false;
};

bool is_query(const std::string& s) {
  size_t i = 0;
  while (i < s.size()) {
    if (isspace(static_cast<unsigned char>(s[i]))) { ++i; continue; }
    if (s.compare(i, 2, "--") == 0) { while (i < s.size() && s[i] != '\n') ++i; continue; }
    break;
  }
  if (i < s.size() && s[i] == '(') return true;
  auto kw = [&](const char* w) {
    size_t k = strlen(w);
    if (s.size() < i + k) return false;
    for (size_t j = 0; j < k; ++j)
      if (tolower(static_cast<unsigned char>(s[i + j])) != w[j]) return false;
    return s.size() == i + k || !isalnum(static_cast<unsigned char>(s[i + k]));
  };
  return kw("select") || kw("with");
}

std::string trim_stmt(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && isspace(static_cast<unsigned char>(s[a]))) ++a;
  while (b > a && (isspace(static_cast<unsigned char>(s[b - 1])) || s[b - 1] == ';')) --b;
  return s.substr(a, b - a);
}

class Gateway {
 public:
  Gateway(std::string host, int port, py::object forward)
      : host_(std::move(host)), port_(port), forward_(std::move(forward)) {
    std::random_device rd;
    rng_.seed((uint64_t(rd()) << 32) ^ rd() ^ static_cast<uint64_t>(now_ms()));
  }
  ~Gateway() { stop(); }

  int start() {
    lfd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    if (lfd_ < 0) throw std::runtime_error("socket() failed");
    int one = 1;
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(static_cast<uint16_t>(port_));
    if (inet_pton(AF_INET, host_.c_str(), &a.sin_addr) != 1) throw std::runtime_error("bad host " + host_);
    if (::bind(lfd_, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0 || ::listen(lfd_, 1024) != 0) {
      ::close(lfd_);
      throw std::runtime_error("bind/listen failed on port " + std::to_string(port_));
    }
    socklen_t len = sizeof a;
    getsockname(lfd_, reinterpret_cast<sockaddr*>(&a), &len);
    port_ = ntohs(a.sin_port);
    running_ = true;
    acceptor_ = std::thread([this] { accept_loop(); });
    return port_;
  }

  void stop() {
    if (!running_.exchange(false)) return;
    ::shutdown(lfd_, SHUT_RDWR);
    ::close(lfd_);
    {
      std::lock_guard<std::mutex> g(mu_);
      for (int fd : conns_) ::shutdown(fd, SHUT_RDWR);
    }
    if (acceptor_.joinable()) acceptor_.join();
    // connection threads exit on their own once their sockets are shut down
    std::unique_lock<std::mutex> lk(mu_);
    conn_cv_.wait_for(lk, std::chrono::seconds(5), [this] { return nconn_ == 0; });
    work_cv_.notify_all();
    done_cv_.notify_all();
  }

  int port() const { return port_; }

  // ---------------------------------------------------------------- Python-facing API
  void set_context(py::bytes sid, int64_t token) {
    std::lock_guard<std::mutex> g(mu_);
    ctx_[std::string(sid)] = token;
  }

  void drop_context(py::bytes sid) {
    std::string s(sid);
    std::lock_guard<std::mutex> g(mu_);
    ctx_.erase(s);
    for (auto it = ops_.begin(); it != ops_.end();) {
      if (it->second.sid == s) {
        release_op(it->second);
        it = ops_.erase(it);
      } else {
        ++it;
      }
    }
  }

  py::object next_batch(double timeout_s) {
    std::shared_ptr<Batch> b;
    double waited = 0.0;
    {
      py::gil_scoped_release nogil;
      std::unique_lock<std::mutex> lk(mu_);
      work_cv_.wait_for(lk, std::chrono::duration<double>(timeout_s),
                        [this] { return !queue_.empty() || !running_; });
      while (!queue_.empty()) {
        b = queue_.front();
        queue_.pop_front();
        if (pending_.count(b->key) && pending_[b->key] == b) pending_.erase(b->key);
        if (b->live == 0 || (b->cancels >= b->live)) {  // every waiter left or cancelled
          running_batches_.erase(b->id);
          b->state = OP_CANCELED;
          b->completed = now_ms();
          b.reset();
          continue;
        }
        b->state = OP_RUNNING;
        b->started = now_ms();
        waited = steady_s() - b->queued_at;
        ++stats_batches_;
        break;
      }
    }
    if (!b) return py::none();
    // (id, session, statement, seconds the batch waited in the admission queue)
    return py::make_tuple(b->id, py::bytes(b->sid), b->stmt, waited);
  }

  void finish_batch(int64_t id, py::bytes schema, py::list cols, int64_t nrows, py::object error) {
    std::vector<Col> cv;
    if (error.is_none()) {
      for (auto item : cols) {
        py::tuple t = item.cast<py::tuple>();
        Col c;
        c.kind = t[0].cast<int>();
        c.data = t[1].cast<std::string>();
        std::string offs = t[2].cast<std::string>();
        c.nulls = t[3].cast<std::string>();
        if (c.kind == 6) {
          c.off.resize(offs.size() / 8);
          std::memcpy(c.off.data(), offs.data(), c.off.size() * 8);
          if (static_cast<int64_t>(c.off.size()) != nrows + 1) throw std::runtime_error("bad string offsets");
        } else {
          static const int width[] = {1, 1, 2, 4, 8, 8};
          if (c.kind < 0 || c.kind > 5 || static_cast<int64_t>(c.data.size()) != nrows * width[c.kind])
            throw std::runtime_error("bad column payload");
        }
        if (static_cast<int64_t>(c.nulls.size()) != nrows) throw std::runtime_error("bad null mask");
        cv.push_back(std::move(c));
      }
    }
    std::string sch(schema);
    std::string err = error.is_none() ? std::string() : error.cast<std::string>();
    py::gil_scoped_release nogil;
    std::lock_guard<std::mutex> g(mu_);
    auto it = running_batches_.find(id);
    if (it == running_batches_.end()) return;
    auto b = it->second;
    running_batches_.erase(it);
    b->schema = std::move(sch);
    b->cols = std::move(cv);
    b->nrows = nrows;
    b->error = err;
    b->state = err.empty() ? OP_FINISHED : OP_ERROR;
    b->completed = now_ms();
    done_cv_.notify_all();
  }

  // identical queued statements execute once (on by default); off measures engine throughput
  void set_coalesce(bool on) {
    std::lock_guard<std::mutex> g(mu_);
    coalesce_ = on;
  }

  bool is_cancelled(int64_t id) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = running_batches_.find(id);
    return it == running_batches_.end() || it->second->cancel;
  }

  py::dict stats() {
    std::lock_guard<std::mutex> g(mu_);
    py::dict d;
    d["statements"] = stats_statements_;
    d["batches"] = stats_batches_;
    d["coalesced"] = stats_coalesced_;
    d["forwarded"] = stats_forwarded_;
    d["connections"] = nconn_;
    d["open_ops"] = static_cast<int64_t>(ops_.size());
    return d;
  }

 private:
  // ---------------------------------------------------------------- connection handling
  void accept_loop() {
    while (running_) {
      int fd = ::accept(lfd_, nullptr, nullptr);
      if (fd < 0) {
        if (!running_) break;
        continue;
      }
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      {
        std::lock_guard<std::mutex> g(mu_);
        conns_.insert(fd);
        ++nconn_;
      }
      std::thread([this, fd] { serve(fd); }).detach();
    }
  }

  struct Sock {
    int fd;
    std::string buf;
    size_t pos = 0;
    bool fill(size_t want) {  // make buf[pos, pos+want) available
      while (buf.size() - pos < want) {
        if (pos > 0 && pos == buf.size()) { buf.clear(); pos = 0; }
        char tmp[65536];
        ssize_t k = ::recv(fd, tmp, sizeof tmp, 0);
        if (k <= 0) return false;
        buf.append(tmp, static_cast<size_t>(k));
      }
      return true;
    }
    bool read(size_t n, std::string& out) {
      if (!fill(n)) return false;
      out.assign(buf, pos, n);
      pos += n;
      return true;
    }
    bool peek1(uint8_t& c) {
      if (!fill(1)) return false;
      c = static_cast<uint8_t>(buf[pos]);
      return true;
    }
    bool send_all(const std::string& s) {
      size_t o = 0;
      while (o < s.size()) {
        ssize_t k = ::send(fd, s.data() + o, s.size() - o, MSG_NOSIGNAL);
        if (k <= 0) return false;
        o += static_cast<size_t>(k);
      }
      return true;
    }
  };

  static int32_t be32(const std::string& s, size_t o = 0) {
    const auto* p = reinterpret_cast<const uint8_t*>(s.data() + o);
    return static_cast<int32_t>((uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3]);
  }

  // one unframed binary-protocol message: header + args struct (skipped to find its end)
  bool read_unframed(Sock& s, std::string& msg) {
    msg.clear();
    std::string t;
    auto take = [&](size_t n) -> bool {
      if (!s.read(n, t)) return false;
      msg += t;
      return true;
    };
    std::function<bool(int8_t, int)> skip = [&](int8_t ty, int depth) -> bool {
      if (depth > 64) return false;
      switch (ty) {
        case T_BOOL: case T_BYTE: return take(1);
        case T_I16: return take(2);
        case T_I32: return take(4);
        case T_I64: case T_DOUBLE: return take(8);
        case T_STRING: {
          if (!take(4)) return false;
          int32_t n = be32(msg, msg.size() - 4);
          return n >= 0 && take(static_cast<size_t>(n));
        }
        case T_STRUCT:
          for (;;) {
            if (!take(1)) return false;
            int8_t ft = static_cast<int8_t>(msg.back());
            if (ft == T_STOP) return true;
            if (!take(2) || !skip(ft, depth + 1)) return false;
          }
        case T_LIST: case T_SET: {
          if (!take(5)) return false;
          int8_t et = static_cast<int8_t>(msg[msg.size() - 5]);
          int32_t n = be32(msg, msg.size() - 4);
          for (int32_t j = 0; j < n; ++j)
            if (!skip(et, depth + 1)) return false;
          return n >= 0;
        }
        case T_MAP: {
          if (!take(6)) return false;
          int8_t kt = static_cast<int8_t>(msg[msg.size() - 6]), vt = static_cast<int8_t>(msg[msg.size() - 5]);
          int32_t n = be32(msg, msg.size() - 4);
          for (int32_t j = 0; j < n; ++j)
            if (!skip(kt, depth + 1) || !skip(vt, depth + 1)) return false;
          return n >= 0;
        }
        default: return false;
      }
    };
    if (!take(4)) return false;
    int32_t v = be32(msg, 0);
    if (v < 0) {
      if (!take(4)) return false;
      int32_t n = be32(msg, 4);
      if (n < 0 || !take(static_cast<size_t>(n)) || !take(4)) return false;
    } else {
      if (!take(static_cast<size_t>(v)) || !take(1) || !take(4)) return false;
    }
    return skip(T_STRUCT, 0);
  }

  void serve(int fd) {
    Sock s{fd, std::string(), 0};
    try {
      uint8_t first;
      if (s.peek1(first)) {
        bool framed = false;
        if (first == SASL_START) {
          if (!sasl(s)) throw ProtocolError("sasl");
          framed = true;
        }
        std::string msg, hdr;
        for (;;) {
          if (framed) {
            if (!s.read(4, hdr)) break;
            int32_t n = be32(hdr);
            if (n < 0 || n > (1 << 30) || !s.read(static_cast<size_t>(n), msg)) break;
          } else if (!read_unframed(s, msg)) {
            break;
          }
          std::string out = dispatch(msg);
          if (framed) {
            W w;
            w.i32(static_cast<int32_t>(out.size()));
            if (!s.send_all(w.b + out)) break;
          } else if (!s.send_all(out)) {
            break;
          }
        }
      }
    } catch (const std::exception&) {
    }
    ::close(fd);
    std::lock_guard<std::mutex> g(mu_);
    conns_.erase(fd);
    --nconn_;
    conn_cv_.notify_all();
  }

  bool sasl(Sock& s) {
    // START: status(1) len(4) mechanism ; then one message with the PLAIN payload "\0user\0password"
    std::string st, ln, mech, payload;
    if (!s.read(1, st) || !s.read(4, ln)) return false;
    int32_t n = be32(ln);
    if (n < 0 || !s.read(static_cast<size_t>(n), mech)) return false;
    for (auto& c : mech) c = static_cast<char>(toupper(static_cast<unsigned char>(c)));
    if (mech != "PLAIN" && mech != "ANONYMOUS") {
      std::string bad(1, static_cast<char>(SASL_BAD));
      bad += std::string(4, '\0');
      s.send_all(bad);
      return false;
    }
    if (!s.read(1, st) || !s.read(4, ln)) return false;
    n = be32(ln);
    if (n < 0 || !s.read(static_cast<size_t>(n), payload)) return false;
    std::string ok(1, static_cast<char>(SASL_COMPLETE));
    ok += std::string(4, '\0');
    return s.send_all(ok);
  }

  // ---------------------------------------------------------------- RPC dispatch
  std::string dispatch(const std::string& msg) {
    std::string name;
    int32_t seqid = 0;
    Node args;
    try {
      R r(msg);
      int32_t v = r.i32();
      if (v < 0) {
        if ((static_cast<uint32_t>(v) & 0xffff0000u) != VERSION_1) throw ProtocolError("bad version");
        name = r.str();
        seqid = r.i32();
      } else {
        r.need(static_cast<size_t>(v));
        name.assign(reinterpret_cast<const char*>(r.p + r.o), static_cast<size_t>(v));
        r.o += static_cast<size_t>(v);
        r.i8();
        seqid = r.i32();
      }
      read_value(r, T_STRUCT, args);
    } catch (const std::exception&) {
      return forward(msg);
    }
    const Node* req = args.get(1);
    if (req == nullptr || req->t != T_STRUCT) return forward(msg);
    if (name == "ExecuteStatement") return execute(msg, *req, seqid);
    if (name == "GetOperationStatus" || name == "GetResultSetMetadata" || name == "FetchResults" ||
        name == "CloseOperation" || name == "CancelOperation")
      return op_call(msg, name, *req, seqid);
    return forward(msg);
  }

  std::string forward(const std::string& msg) {
    {
      std::lock_guard<std::mutex> g(mu_);
      ++stats_forwarded_;
    }
    py::gil_scoped_acquire gil;
    py::object r = forward_(py::bytes(msg));
    return r.cast<std::string>();
  }

  static void status_ok(W& w) {
    w.field(T_STRUCT, 1);
    w.field(T_I32, 1);
    w.i32(0);
    w.stop();
  }

  static void status_err(W& w, const std::string& m, int16_t fid = 1) {
    w.field(T_STRUCT, fid);
    w.field(T_I32, 1);
    w.i32(3);  // ERROR_STATUS
    w.field(T_STRING, 3);
    w.str("42000");
    w.field(T_I32, 4);
    w.i32(0);
    w.field(T_STRING, 5);
    w.str(m.empty() ? std::string("error") : m);
    w.stop();
  }

  static void handle_struct(W& w, int16_t fid, const std::string& guid, const std::string& secret) {
    w.field(T_STRUCT, fid);
    w.field(T_STRUCT, 1);  // operationId
    w.field(T_STRING, 1);
    w.str(guid);
    w.field(T_STRING, 2);
    w.str(secret);
    w.stop();
    w.field(T_I32, 2);  // operationType EXECUTE_STATEMENT
    w.i32(0);
    w.field(T_BOOL, 3);  // hasResultSet
    w.i8(1);
    w.stop();
  }

  std::string random_guid() {
    std::string g(16, '\0');
    for (int i = 0; i < 16; i += 8) {
      uint64_t x = rng_();
      std::memcpy(&g[i], &x, 8);
    }
    return g;
  }

  std::string execute(const std::string& msg, const Node& req, int32_t seqid) {
    const Node* sh = req.get(1);
    const Node* st = req.get(2);
    const Node* overlay = req.get(3);
    const Node* tmo = req.get(5);
    const Node* sidn = sh ? sh->get(1) : nullptr;
    const Node* guid = sidn ? sidn->get(1) : nullptr;
    if (!guid || !st || (overlay && overlay->nlist > 0) || (tmo && tmo->i > 0)) return forward(msg);
    std::string stmt = trim_stmt(st->s);
    if (!is_query(stmt)) return forward(msg);
    const Node* ra = req.get(4);
    bool async = ra && ra->i != 0;
    std::shared_ptr<Batch> b;
    std::string opid, secret;
    {
      std::unique_lock<std::mutex> g(mu_);
      auto cit = ctx_.find(guid->s);
      if (cit == ctx_.end()) {  // no published context yet: the Python server decides
        g.unlock();
        return forward(msg);
      }
      std::string key = std::to_string(cit->second) + '\x1f' + stmt;
      ++stats_statements_;
      auto pit = pending_.find(key);
      // a queued batch whose waiters all cancelled (or left) keeps its sticky cancel flag: a new
      // statement must not join it, or it would be reported 'cancelled' without ever cancelling
      if (coalesce_ && pit != pending_.end() && !pit->second->cancel) {
        b = pit->second;
        ++stats_coalesced_;
      } else {
        b = std::make_shared<Batch>();
        b->id = ++next_batch_;
        b->sid = guid->s;
        b->stmt = stmt;
        b->key = key;
        b->queued_at = steady_s();
        pending_[key] = b;
        queue_.push_back(b);
        running_batches_[b->id] = b;
        work_cv_.notify_one();
      }
      ++b->live;
      opid = random_guid();
      secret = random_guid();
      Op op;
      op.b = b;
      op.secret = secret;
      op.sid = guid->s;
      ops_[opid] = std::move(op);
    }
    W w;
    w.msg("ExecuteStatement", seqid);
    w.field(T_STRUCT, 0);
    if (!async) {
      std::unique_lock<std::mutex> lk(mu_);
      done_cv_.wait(lk, [&] { return b->state >= OP_FINISHED || !running_; });
      if (b->state == OP_ERROR || b->state == OP_CANCELED) {
        std::string err = b->state == OP_ERROR ? b->error : std::string("cancelled");
        auto it = ops_.find(opid);
        if (it != ops_.end()) {
          release_op(it->second);
          ops_.erase(it);
        }
        lk.unlock();
        status_err(w, err);
        w.stop();
        w.stop();
        return w.b;
      }
    }
    status_ok(w);
    handle_struct(w, 2, opid, secret);
    w.stop();
    w.stop();
    return w.b;
  }

  void release_op(Op& op) {  // mu_ held
    if (!op.b) return;
    --op.b->live;
    if (op.cancelled) --op.b->cancels;
    if (op.b->state <= OP_RUNNING && op.b->live > 0 && op.b->cancels >= op.b->live) op.b->cancel = true;
    if (op.b->live <= 0 && op.b->state <= OP_RUNNING) op.b->cancel = true;
    op.b.reset();
  }

  std::string op_call(const std::string& msg, const std::string& name, const Node& req, int32_t seqid) {
    const Node* oh = req.get(1);
    const Node* oid = oh ? oh->get(1) : nullptr;
    const Node* g = oid ? oid->get(1) : nullptr;
    if (!g) return forward(msg);
    W w;
    w.msg(name, seqid);
    w.field(T_STRUCT, 0);
    std::unique_lock<std::mutex> lk(mu_);
    auto it = ops_.find(g->s);
    if (it == ops_.end()) {
      lk.unlock();
      return forward(msg);  // a Python-owned operation (commands, metadata calls)
    }
    Op& op = it->second;
    std::shared_ptr<Batch> b = op.b;
    if (name == "CloseOperation") {
      release_op(op);
      ops_.erase(it);
      lk.unlock();
      status_ok(w);
    } else if (name == "CancelOperation") {
      if (!op.cancelled) {
        op.cancelled = true;
        ++b->cancels;
        if (b->state <= OP_RUNNING && b->cancels >= b->live) b->cancel = true;
      }
      lk.unlock();
      status_ok(w);
    } else if (name == "GetOperationStatus") {
      int state = op.cancelled ? OP_CANCELED : (b->state == OP_INITIALIZED ? OP_RUNNING : b->state);
      std::string err = b->error;
      int64_t started = b->started, completed = b->completed;
      lk.unlock();
      status_ok(w);
      w.field(T_I32, 2);
      w.i32(state);
      if (state == OP_ERROR) {
        w.field(T_STRING, 3);
        w.str("42000");
        w.field(T_I32, 4);
        w.i32(0);
        w.field(T_STRING, 5);
        w.str(err);
      }
      w.field(T_I64, 7);
      w.i64(started);
      w.field(T_I64, 8);
      w.i64(completed);
      w.field(T_BOOL, 9);
      w.i8(1);
    } else {  // GetResultSetMetadata / FetchResults: wait for the batch
      done_cv_.wait(lk, [&] { return b->state >= OP_FINISHED || op.cancelled || !running_; });
      if (b->state != OP_FINISHED || op.cancelled) {
        std::string err = op.cancelled || b->state == OP_CANCELED ? std::string("cancelled") : b->error;
        lk.unlock();
        status_err(w, err);
      } else if (name == "GetResultSetMetadata") {
        lk.unlock();
        status_ok(w);
        w.field(T_STRUCT, 2);
        w.b += b->schema;  // already a complete TTableSchema struct (fields + STOP)
      } else {
        const Node* ori = req.get(2);
        const Node* mr = req.get(3);
        const Node* ft = req.get(4);
        if (ft && ft->i == 1) {  // operation log: empty
          lk.unlock();
          status_ok(w);
          w.field(T_BOOL, 2);
          w.i8(0);
          w.field(T_STRUCT, 3);
          w.field(T_I64, 1);
          w.i64(0);
          w.field(T_LIST, 2);
          w.i8(T_STRUCT);
          w.i32(0);
          w.field(T_LIST, 3);
          w.i8(T_STRUCT);
          w.i32(0);
          w.stop();
        } else {
          if (ori && ori->i == 4) op.cursor = 0;  // FETCH_FIRST
          int64_t n = (mr && mr->i > 0) ? mr->i : 1000;
          int64_t a = op.cursor, e = std::min(b->nrows, op.cursor + n);
          op.cursor = e;
          lk.unlock();  // the batch's columns are immutable once finished
          status_ok(w);
          w.field(T_BOOL, 2);
          w.i8(e < b->nrows ? 1 : 0);
          w.field(T_STRUCT, 3);
          w.field(T_I64, 1);
          w.i64(a);
          w.field(T_LIST, 2);
          w.i8(T_STRUCT);
          w.i32(0);
          w.field(T_LIST, 3);
          w.i8(T_STRUCT);
          w.i32(static_cast<int32_t>(b->cols.size()));
          for (const Col& c : b->cols) write_column(w, c, a, e);
          w.stop();
        }
      }
    }
    w.stop();
    w.stop();
    return w.b;
  }

  static void write_column(W& w, const Col& c, int64_t a, int64_t e) {
    static const int8_t elem[] = {T_BOOL, T_BYTE, T_I16, T_I32, T_I64, T_DOUBLE, T_STRING};
    static const int width[] = {1, 1, 2, 4, 8, 8};
    w.field(T_STRUCT, static_cast<int16_t>(c.kind + 1));  // TColumn union member
    w.field(T_LIST, 1);
    w.i8(elem[c.kind]);
    int64_t n = e - a;
    w.i32(static_cast<int32_t>(n));
    const char* d = c.data.data();
    for (int64_t i = a; i < e; ++i) {
      switch (c.kind) {
        case 0: case 1: w.i8(static_cast<int8_t>(d[i])); break;
        case 2: { int16_t v; std::memcpy(&v, d + i * 2, 2); w.i16(v); break; }
        case 3: { int32_t v; std::memcpy(&v, d + i * 4, 4); w.i32(v); break; }
        case 4: { int64_t v; std::memcpy(&v, d + i * 8, 8); w.i64(v); break; }
        case 5: { double v; std::memcpy(&v, d + i * 8, 8); w.dbl(v); break; }
        default: w.str(d + c.off[i], static_cast<size_t>(c.off[i + 1] - c.off[i]));
      }
    }
    (void)width;
    // nulls: bit i of the slice set = row a+i is NULL (LSB first)
    std::string bits(static_cast<size_t>((n + 7) / 8), '\0');
    for (int64_t i = 0; i < n; ++i)
      if (c.nulls[static_cast<size_t>(a + i)]) bits[static_cast<size_t>(i / 8)] |= static_cast<char>(1 << (i % 8));
    w.field(T_STRING, 2);
    w.str(bits);
    w.stop();
    w.stop();
  }

  std::string host_;
  int port_;
  py::object forward_;
  int lfd_ = -1;
  std::atomic<bool> running_{false};
  std::thread acceptor_;
  std::mutex mu_;
  std::condition_variable work_cv_, done_cv_, conn_cv_;
  std::set<int> conns_;
  int64_t nconn_ = 0;
  std::unordered_map<std::string, int64_t> ctx_;
  std::unordered_map<std::string, std::shared_ptr<Batch>> pending_;
  std::unordered_map<int64_t, std::shared_ptr<Batch>> running_batches_;
  std::deque<std::shared_ptr<Batch>> queue_;
  std::unordered_map<std::string, Op> ops_;
  int64_t next_batch_ = 0;
  bool coalesce_ = true;
  int64_t stats_statements_ = 0, stats_batches_ = 0, stats_coalesced_ = 0, stats_forwarded_ = 0;
  std::mt19937_64 rng_;
};

}  // namespace

PYBIND11_MODULE(_sdo_gateway, m) {
  m.doc() = "Native HiveServer2 Thrift gateway (connection I/O, protocol, statement batching)";
  py::class_<Gateway>(m, "Gateway")
      .def(py::init<std::string, int, py::object>(), py::arg("host"), py::arg("port"), py::arg("forward"))
      .def("start", &Gateway::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &Gateway::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &Gateway::port)
      .def("set_context", &Gateway::set_context)
      .def("drop_context", &Gateway::drop_context)
      .def("next_batch", &Gateway::next_batch)
      .def("finish_batch", &Gateway::finish_batch)
      .def("is_cancelled", &Gateway::is_cancelled)
      .def("set_coalesce", &Gateway::set_coalesce)
      .def("stats", &Gateway::stats);
}
