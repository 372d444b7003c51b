// Multi-threaded libsvm reader (no GIL) -> CSR batches.
//
// Reference: Sample.parse_line_libsvm / format_samples_sparse and the
// LoadDataThread file-strided thread pool (lr2.py:51-155,232-258): per-line
// Bernoulli sampling `random() < 1 - rate -> skip`, lines shorter than 2 chars
// skipped, `label idx:val ...` split on space/tab.  The reference parses in
// GIL-bound Python threads; here each thread parses its strided share of the
// files natively and the result is CSR (labels, row_ptr, ids, vals) that feeds
// the embedding-bag kernels directly.  A streaming mode (queue semantics of
// lr2.py --mode=queue) pushes fixed-size batches through a bounded queue and
// can loop over the files forever like the reference loaders (A9).
#include <torch/extension.h>
#include <pybind11/numpy.h>

#include <atomic>
#include <condition_variable>

#include "cv_wait.h"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace dtf {
namespace libsvm {

struct CSR {
  std::vector<float> labels;
  std::vector<int64_t> row_ptr{0};
  std::vector<int64_t> ids;
  std::vector<float> vals;
  int64_t rows() const { return (int64_t)labels.size(); }
  void append(const CSR& o) {
    const int64_t base = (int64_t)ids.size();
    labels.insert(labels.end(), o.labels.begin(), o.labels.end());
    for (size_t i = 1; i < o.row_ptr.size(); ++i) row_ptr.push_back(base + o.row_ptr[i]);
    ids.insert(ids.end(), o.ids.begin(), o.ids.end());
    vals.insert(vals.end(), o.vals.begin(), o.vals.end());
  }
};

struct Rng {  // xorshift64*
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0x2545F4914F6CDD1Dull) {
    if (!s) s = 1;
  }
  double uniform() {
    s ^= s >> 12; s ^= s << 25; s ^= s >> 27;
    return (double)((s * 2685821657736338717ull) >> 11) * (1.0 / 9007199254740992.0);
  }
};

// Parses one line [p, e). Returns false for a malformed line.
static bool parse_line(const char* p, const char* e, CSR& out) {
  auto skip_ws = [&] { while (p < e && (*p == ' ' || *p == '\t' || *p == '\r')) ++p; };
  skip_ws();
  if (p >= e) return false;
  char* end = nullptr;
  std::string tmp;
  const float label = strtof(p, &end);
  if (end == p) return false;
  p = end;
  const size_t nnz0 = out.ids.size();
  while (true) {
    skip_ws();
    if (p >= e) break;
    const long long idx = strtoll(p, &end, 10);
    if (end == p || end >= e || *end != ':') {
      out.ids.resize(nnz0);
      out.vals.resize(nnz0);
      return false;
    }
    p = end + 1;
    const float v = strtof(p, &end);
    if (end == p) {
      out.ids.resize(nnz0);
      out.vals.resize(nnz0);
      return false;
    }
    p = end;
    out.ids.push_back(idx);
    out.vals.push_back(v);
  }
  out.labels.push_back(label);
  out.row_ptr.push_back((int64_t)out.ids.size());
  return true;
}

// Parse a whole buffer; sampling with rate (1.0 keeps all).
static void parse_buffer(const char* data, size_t n, double rate, Rng& rng, CSR& out,
                         int64_t* bad_lines) {
  const char* p = data;
  const char* end = data + n;
  // strtof/strtoll need a terminator after the last number: lines are parsed
  // in-place, every line ends at '\n' or at `end` (the caller NUL-pads).
  while (p < end) {
    const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
    const char* le = nl ? nl : end;
    if (le - p >= 2 && !(rng.uniform() < 1.0 - rate)) {
      if (!parse_line(p, le, out) && bad_lines) ++*bad_lines;
    }
    p = nl ? nl + 1 : end;
  }
}

static std::string read_file(const std::string& path) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open " + path);
  std::string s;
  char buf[1 << 16];
  size_t k;
  while ((k = fread(buf, 1, sizeof(buf), f)) > 0) s.append(buf, k);
  fclose(f);
  s.push_back('\0');
  return s;
}

template <typename T>
static py::array_t<T> to_np(std::vector<T>&& v) {
  auto* heap = new std::vector<T>(std::move(v));
  py::capsule owner(heap, [](void* p) { delete reinterpret_cast<std::vector<T>*>(p); });
  return py::array_t<T>({(py::ssize_t)heap->size()}, {(py::ssize_t)sizeof(T)}, heap->data(), owner);
}

static py::tuple to_py(CSR&& c) {
  return py::make_tuple(to_np(std::move(c.labels)), to_np(std::move(c.row_ptr)), to_np(std::move(c.ids)),
                        to_np(std::move(c.vals)));
}

py::tuple parse_bytes(py::bytes data, double rate, uint64_t seed) {
  std::string s = data;
  s.push_back('\0');
  CSR out;
  int64_t bad = 0;
  {
    py::gil_scoped_release nogil;
    Rng rng(seed);
    parse_buffer(s.data(), s.size() - 1, rate, rng, out, &bad);
  }
  return to_py(std::move(out));
}

// thread t parses files[t::nthreads] (reference InitThreads striding); the
// per-thread results are concatenated in thread order (LoadDataAll).
py::tuple parse_files(std::vector<std::string> files, int nthreads, double rate, uint64_t seed) {
  if (nthreads < 1) nthreads = 1;
  std::vector<CSR> parts(nthreads);
  std::vector<std::string> errs(nthreads);
  {
    py::gil_scoped_release nogil;
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) {
      th.emplace_back([&, t] {
        try {
          Rng rng(seed + 7919ull * t);
          for (size_t i = t; i < files.size(); i += nthreads) {
            std::string s = read_file(files[i]);
            parse_buffer(s.data(), s.size() - 1, rate, rng, parts[t], nullptr);
          }
        } catch (std::exception& e) {
          errs[t] = e.what();
        }
      });
    }
    for (auto& x : th) x.join();
  }
  for (auto& e : errs) if (!e.empty()) throw std::runtime_error(e);
  CSR all;
  for (auto& p : parts) all.append(p);
  return to_py(std::move(all));
}

// Streaming reader: producer threads parse strided files and emit batches of
// `batch` rows through a bounded queue (capacity in batches); loop=true wraps
// around the file list forever (reference queue mode).
class Stream {
 public:
  Stream(std::vector<std::string> files, int64_t batch, int nthreads, double rate, bool loop,
         int capacity, uint64_t seed)
      : files_(std::move(files)), batch_(batch), rate_(rate), loop_(loop), cap_(capacity) {
    if (batch <= 0) throw std::invalid_argument("batch must be positive");
    if (nthreads < 1) nthreads = 1;
    live_ = nthreads;
    for (int t = 0; t < nthreads; ++t) th_.emplace_back([this, t, nthreads, seed] { run(t, nthreads, seed); });
  }
  ~Stream() { stop(); }
  void stop() {
    std::lock_guard<std::mutex> g(stop_mu_);   // one joiner at a time
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      cv_.notify_all();
    }
    for (auto& t : th_) if (t.joinable()) t.join();
    th_.clear();
  }
  // returns None when all producers finished and the queue is drained
  py::object next(double timeout) {
    CSR b;
    bool done = false;
    {
      py::gil_scoped_release nogil;
      std::unique_lock<std::mutex> lk(mu_);
      auto pred = [&] { return !q_.empty() || live_ == 0 || !err_.empty(); };
      if (timeout < 0) cv_.wait(lk, pred);
      else if (!cv_wait_for(cv_, lk, std::chrono::duration<double>(timeout), pred))
        throw std::runtime_error("libsvm stream timed out");
      if (!err_.empty()) throw std::runtime_error(err_);
      if (q_.empty()) {
        done = true;
      } else {
        b = std::move(q_.front());
        q_.pop_front();
        cv_.notify_all();
      }
    }
    if (done) return py::none();
    return to_py(std::move(b));
  }
  int64_t rows_emitted() const { return emitted_.load(); }

 private:
  void push(CSR&& b) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return stop_ || (int)q_.size() < cap_; });
    if (stop_) return;
    emitted_ += b.rows();
    q_.push_back(std::move(b));
    cv_.notify_all();
  }
  void run(int t, int n, uint64_t seed) {
    try {
      Rng rng(seed + 104729ull * t);
      CSR cur;
      do {
        bool any = false;
        for (size_t i = t; i < files_.size(); i += n) {
          any = true;
          std::string s = read_file(files_[i]);
          CSR part;
          parse_buffer(s.data(), s.size() - 1, rate_, rng, part, nullptr);
          // slice into batches (carry the remainder to the next file)
          for (int64_t r = 0; r < part.rows(); ++r) {
            cur.labels.push_back(part.labels[r]);
            for (int64_t k = part.row_ptr[r]; k < part.row_ptr[r + 1]; ++k) {
              cur.ids.push_back(part.ids[k]);
              cur.vals.push_back(part.vals[k]);
            }
            cur.row_ptr.push_back((int64_t)cur.ids.size());
            if (cur.rows() == batch_) {
              push(std::move(cur));
              cur = CSR();
              if (stopped()) return;
            }
          }
          if (stopped()) return;
        }
        if (!any) break;
      } while (loop_ && !stopped());
      if (cur.rows() > 0 && !stopped()) push(std::move(cur));
    } catch (std::exception& e) {
      std::lock_guard<std::mutex> lk(mu_);
      err_ = e.what();
    }
    std::lock_guard<std::mutex> lk(mu_);
    --live_;
    cv_.notify_all();
  }
  bool stopped() {
    std::lock_guard<std::mutex> lk(mu_);
    return stop_;
  }

  std::vector<std::string> files_;
  int64_t batch_;
  double rate_;
  bool loop_;
  int cap_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<CSR> q_;
  int live_ = 0;
  bool stop_ = false;
  std::string err_;
  std::atomic<int64_t> emitted_{0};
  std::mutex stop_mu_;
  std::vector<std::thread> th_;
};

}  // namespace libsvm

void init_libsvm(py::module& m) {
  using namespace libsvm;
  m.def("libsvm_parse_bytes", &parse_bytes, py::arg("data"), py::arg("sampling_rate") = 1.0,
        py::arg("seed") = 0);
  m.def("libsvm_parse_files", &parse_files, py::arg("files"), py::arg("nthreads") = 2,
        py::arg("sampling_rate") = 1.0, py::arg("seed") = 0);
  py::class_<Stream>(m, "LibsvmStream")
      .def(py::init<std::vector<std::string>, int64_t, int, double, bool, int, uint64_t>(),
           py::arg("files"), py::arg("batch_size"), py::arg("nthreads") = 2,
           py::arg("sampling_rate") = 1.0, py::arg("loop") = false, py::arg("capacity") = 8,
           py::arg("seed") = 0)
      .def("next", &Stream::next, py::arg("timeout") = -1.0)
      .def("stop", &Stream::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("rows_emitted", &Stream::rows_emitted);
}

}  // namespace dtf
