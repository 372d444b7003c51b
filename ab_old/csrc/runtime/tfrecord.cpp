// TFRecord framing + asynchronous tfevents writer (TensorBoard event files).
//
// Reference behaviour: `tf.train.SummaryWriter(logs_path, graph)` and
// `writer.add_summary(summary, step)` on every step (example.py:154,171).
// Each record is  u64 len | u32 masked_crc32c(len) | data | u32 masked_crc32c(data).
// Events are serialized `Event` protos (wall_time=1, step=2, file_version=3,
// graph_def=4, summary=5; Summary.Value tag=1 simple_value=2 histo=5).
//
// Writes go through a background thread so that a per-step summary never
// blocks the training loop (the reference pays a synchronous file append per
// step).
#include <torch/extension.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>

#include "cv_wait.h"
#include <cstdio>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "crc32c.h"
#include "wire.h"

namespace dtf {

static std::string frame_record(const std::string& data) {
  std::string out;
  out.reserve(data.size() + 16);
  uint64_t len = data.size();
  char lb[8];
  memcpy(lb, &len, 8);
  out.append(lb, 8);
  wire::put_fixed32(out, crc32c_mask(crc32c(lb, 8)));
  out.append(data);
  wire::put_fixed32(out, crc32c_mask(crc32c(data.data(), data.size())));
  return out;
}

// Returns all records of a TFRecord file; throws on a CRC mismatch.
static std::vector<py::bytes> read_records(const std::string& path, bool check_crc) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open " + path);
  std::vector<py::bytes> out;
  while (true) {
    char hdr[12];
    size_t n = fread(hdr, 1, 12, f);
    if (n == 0) break;
    if (n != 12) { fclose(f); throw std::runtime_error("truncated record header"); }
    uint64_t len;
    uint32_t lcrc;
    memcpy(&len, hdr, 8);
    memcpy(&lcrc, hdr + 8, 4);
    if (check_crc && crc32c_mask(crc32c(hdr, 8)) != lcrc) {
      fclose(f);
      throw std::runtime_error("record length CRC mismatch");
    }
    std::string data(len, '\0');
    uint32_t dcrc;
    if (fread(&data[0], 1, len, f) != len || fread(&dcrc, 1, 4, f) != 4) {
      fclose(f);
      throw std::runtime_error("truncated record");
    }
    if (check_crc && crc32c_mask(crc32c(data.data(), data.size())) != dcrc) {
      fclose(f);
      throw std::runtime_error("record data CRC mismatch");
    }
    out.emplace_back(data);
  }
  fclose(f);
  return out;
}

static std::string encode_scalar_event(double wall_time, int64_t step, const std::string& tag,
                                       float value) {
  std::string val, summ, ev;
  wire::put_bytes(val, 1, tag);
  wire::put_float(val, 2, value);
  wire::put_bytes(summ, 1, val);
  wire::put_double(ev, 1, wall_time);
  wire::put_int(ev, 2, step);
  wire::put_bytes(ev, 5, summ);
  return ev;
}

static std::string encode_histo_value(const std::string& tag, const std::vector<double>& values,
                                      int nbuckets) {
  double mn = 0, mx = 0, sum = 0, sq = 0;
  if (!values.empty()) {
    mn = mx = values[0];
    for (double v : values) {
      mn = std::min(mn, v);
      mx = std::max(mx, v);
      sum += v;
      sq += v * v;
    }
  }
  std::vector<double> limits, counts;
  if (nbuckets < 1) nbuckets = 1;
  double w = (mx - mn) / nbuckets;
  if (w <= 0) w = 1.0;
  for (int i = 0; i < nbuckets; ++i) limits.push_back(i == nbuckets - 1 ? 1.7976931348623157e308 : mn + w * (i + 1));
  counts.assign(nbuckets, 0.0);
  for (double v : values) {
    int b = (int)((v - mn) / w);
    if (b >= nbuckets) b = nbuckets - 1;
    if (b < 0) b = 0;
    counts[b] += 1.0;
  }
  std::string h;
  wire::put_double(h, 1, mn);
  wire::put_double(h, 2, mx);
  wire::put_double(h, 3, (double)values.size());
  wire::put_double(h, 4, sum);
  wire::put_double(h, 5, sq);
  std::string packed;
  for (double l : limits) { uint64_t u; memcpy(&u, &l, 8); wire::put_fixed64(packed, u); }
  wire::put_bytes(h, 6, packed);
  packed.clear();
  for (double c : counts) { uint64_t u; memcpy(&u, &c, 8); wire::put_fixed64(packed, u); }
  wire::put_bytes(h, 7, packed);
  std::string val;
  wire::put_bytes(val, 1, tag);
  wire::put_bytes(val, 5, h);
  return val;
}

class EventFileWriter {
 public:
  EventFileWriter(const std::string& path, double flush_secs, int max_queue)
      : path_(path), flush_secs_(flush_secs), max_queue_(max_queue) {
    f_ = fopen(path.c_str(), "ab");
    if (!f_) throw std::runtime_error("cannot open event file " + path);
    std::string ev;
    wire::put_double(ev, 1, now());
    wire::put_bytes(ev, 3, "brain.Event:2");
    push(ev);
    th_ = std::thread([this] { loop(); });
  }
  ~EventFileWriter() { close(); }

  static double now() {
    using namespace std::chrono;
    return duration_cast<duration<double>>(system_clock::now().time_since_epoch()).count();
  }
  void add_event(py::bytes ev) { push(std::string(ev)); }
  void add_scalar(const std::string& tag, double value, int64_t step, double wall_time) {
    push(encode_scalar_event(wall_time > 0 ? wall_time : now(), step, tag, (float)value));
  }
  // summary: a serialized `Summary` proto
  void add_summary(py::bytes summary, int64_t step, double wall_time) {
    std::string ev;
    wire::put_double(ev, 1, wall_time > 0 ? wall_time : now());
    wire::put_int(ev, 2, step);
    wire::put_bytes(ev, 5, std::string(summary));
    push(ev);
  }
  void add_graph(py::bytes graph_def, double wall_time) {
    std::string ev;
    wire::put_double(ev, 1, wall_time > 0 ? wall_time : now());
    wire::put_bytes(ev, 4, std::string(graph_def));
    push(ev);
  }
  void flush() {
    std::unique_lock<std::mutex> lk(mu_);
    flush_req_ = true;
    cv_.notify_all();
    done_cv_.wait(lk, [this] { return q_.empty() && !writing_; });
    if (f_) fflush(f_);
  }
  void close() {
    // serialised so a racing second close (destructor vs. explicit close on
    // another thread) waits for the join instead of leaving th_ joinable
    std::lock_guard<std::mutex> g(close_mu_);
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (closed_) return;
      closed_ = true;
      cv_.notify_all();
    }
    if (th_.joinable()) th_.join();
    if (f_) {
      fflush(f_);
      fclose(f_);
      f_ = nullptr;
    }
  }
  std::string path() const { return path_; }
  int64_t records_written() const { return written_.load(); }

 private:
  void push(std::string ev) {
    std::unique_lock<std::mutex> lk(mu_);
    if (closed_) throw std::runtime_error("event writer closed");
    // bounded queue: the producer only blocks if the disk falls far behind
    done_cv_.wait(lk, [this] { return (int)q_.size() < max_queue_ || closed_; });
    q_.push_back(frame_record(ev));
    cv_.notify_all();
  }
  void loop() {
    auto last_flush = std::chrono::steady_clock::now();
    std::unique_lock<std::mutex> lk(mu_);
    while (true) {
      cv_wait_for(cv_, lk, std::chrono::milliseconds(200),
                  [this] { return !q_.empty() || closed_ || flush_req_; });
      std::deque<std::string> batch;
      batch.swap(q_);
      writing_ = true;
      bool want_flush = flush_req_;
      flush_req_ = false;
      lk.unlock();
      for (auto& r : batch) {
        fwrite(r.data(), 1, r.size(), f_);
        written_++;
      }
      auto t = std::chrono::steady_clock::now();
      if (want_flush || std::chrono::duration<double>(t - last_flush).count() >= flush_secs_) {
        fflush(f_);
        last_flush = t;
      }
      lk.lock();
      writing_ = false;
      done_cv_.notify_all();
      if (closed_ && q_.empty()) break;
    }
  }

  std::string path_;
  double flush_secs_;
  int max_queue_;
  FILE* f_ = nullptr;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::deque<std::string> q_;
  bool closed_ = false, flush_req_ = false, writing_ = false;
  std::atomic<int64_t> written_{0};
  std::mutex close_mu_;
  std::thread th_;
};

void init_tfrecord(py::module& m) {
  m.def("frame_record", [](py::bytes d) { return py::bytes(frame_record(std::string(d))); });
  m.def("read_records", &read_records, py::arg("path"), py::arg("check_crc") = true);
  m.def("write_records", [](const std::string& path, std::vector<py::bytes> recs, bool append) {
    FILE* f = fopen(path.c_str(), append ? "ab" : "wb");
    if (!f) throw std::runtime_error("cannot open " + path);
    for (auto& r : recs) {
      std::string s = frame_record(std::string(r));
      fwrite(s.data(), 1, s.size(), f);
    }
    fclose(f);
  }, py::arg("path"), py::arg("records"), py::arg("append") = false);
  m.def("encode_scalar_event", [](double wt, int64_t step, const std::string& tag, float v) {
    return py::bytes(encode_scalar_event(wt, step, tag, v));
  });
  m.def("encode_histogram_value", [](const std::string& tag, std::vector<double> v, int nb) {
    return py::bytes(encode_histo_value(tag, v, nb));
  });
  m.def("crc32c", [](py::bytes b, uint32_t init) {
    std::string s = b;
    return crc32c_extend(init, s.data(), s.size());
  }, py::arg("data"), py::arg("init") = 0);
  m.def("masked_crc32c", [](py::bytes b) {
    std::string s = b;
    return crc32c_mask(crc32c(s.data(), s.size()));
  });
  m.def("crc32c_hw", &crc32c_hw_available);
  py::class_<EventFileWriter>(m, "EventFileWriter")
      .def(py::init<const std::string&, double, int>(), py::arg("path"), py::arg("flush_secs") = 2.0,
           py::arg("max_queue") = 4096)
      .def("add_event", &EventFileWriter::add_event)
      .def("add_scalar", &EventFileWriter::add_scalar, py::arg("tag"), py::arg("value"),
           py::arg("step"), py::arg("wall_time") = 0.0, py::call_guard<py::gil_scoped_release>())
      .def("add_summary", &EventFileWriter::add_summary, py::arg("summary"), py::arg("step"),
           py::arg("wall_time") = 0.0)
      .def("add_graph", &EventFileWriter::add_graph, py::arg("graph_def"), py::arg("wall_time") = 0.0)
      .def("flush", &EventFileWriter::flush, py::call_guard<py::gil_scoped_release>())
      .def("close", &EventFileWriter::close, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("path", &EventFileWriter::path)
      .def_property_readonly("records_written", &EventFileWriter::records_written);
}

}  // namespace dtf
