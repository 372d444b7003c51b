// Bounded blocking MPMC queue with TF FIFOQueue semantics, natively.
//
// Reference usage: tf.FIFOQueue(capacity=2000) + enqueue_many/dequeue +
// tf.train.batch + close(cancel_pending_enqueues=True) and dequeue timeouts
// (lr2.py:158-175,471-473; input_pipeline_large_dataset.py:18-25,64-65).
// Elements are arbitrary Python objects (tuples of numpy arrays, bytes, ...);
// all waiting happens with the GIL released so producer threads (file readers,
// the libsvm parser) and the training loop run concurrently.
#include <torch/extension.h>

#include <chrono>
#include <condition_variable>

#include "cv_wait.h"
#include <deque>
#include <mutex>
#include <stdexcept>

namespace dtf {

struct QueueClosed : public std::runtime_error {
  QueueClosed() : std::runtime_error("queue closed") {}
};
struct QueueTimeout : public std::runtime_error {
  QueueTimeout() : std::runtime_error("queue operation timed out") {}
};

class BlockingQueue {
 public:
  explicit BlockingQueue(int64_t capacity) : cap_(capacity) {
    if (capacity <= 0) throw std::invalid_argument("capacity must be positive");
  }
  ~BlockingQueue() {
    // drop remaining references (GIL is held by the destructor caller)
    for (PyObject* o : q_) Py_DECREF(o);
  }
  int64_t capacity() const { return cap_; }
  int64_t size() {
    std::lock_guard<std::mutex> lk(mu_);
    return (int64_t)q_.size();
  }
  bool closed() {
    std::lock_guard<std::mutex> lk(mu_);
    return closed_;
  }

  // timeout < 0: wait forever
  void put(py::object item, double timeout) {
    PyObject* o = item.ptr();
    Py_INCREF(o);
    bool ok = false;
    {
      py::gil_scoped_release nogil;
      std::unique_lock<std::mutex> lk(mu_);
      auto pred = [&] { return closed_ || (int64_t)q_.size() < cap_; };
      if (timeout < 0) not_full_.wait(lk, pred);
      else ok = cv_wait_for(not_full_, lk, std::chrono::duration<double>(timeout), pred);
      if (timeout < 0) ok = true;
      if (ok && !closed_) {
        q_.push_back(o);
        not_empty_.notify_one();
        return;
      }
      ok = ok && !closed_;
    }
    Py_DECREF(o);
    if (!ok && closed()) throw QueueClosed();
    throw QueueTimeout();
  }

  // all-or-nothing for the enqueue_many use: blocks until every item is in
  void put_many(py::list items, double timeout) {
    for (auto h : items) put(py::reinterpret_borrow<py::object>(h), timeout);
  }

  py::object get(double timeout) {
    PyObject* o = nullptr;
    bool closed_empty = false;
    {
      py::gil_scoped_release nogil;
      std::unique_lock<std::mutex> lk(mu_);
      auto pred = [&] { return !q_.empty() || closed_; };
      bool ok = true;
      if (timeout < 0) not_empty_.wait(lk, pred);
      else ok = cv_wait_for(not_empty_, lk, std::chrono::duration<double>(timeout), pred);
      if (!q_.empty()) {
        o = q_.front();
        q_.pop_front();
        not_full_.notify_one();
      } else if (closed_) {
        closed_empty = true;
      } else if (!ok) {
        // timeout
      }
    }
    if (o) return py::reinterpret_steal<py::object>(o);
    if (closed_empty) throw QueueClosed();
    throw QueueTimeout();
  }

  py::list get_many(int64_t n, double timeout, bool allow_smaller_final_batch) {
    py::list out;
    for (int64_t i = 0; i < n; ++i) {
      try {
        out.append(get(timeout));
      } catch (QueueClosed&) {
        if (allow_smaller_final_batch && py::len(out) > 0) return out;
        throw;
      }
    }
    return out;
  }

  // cancel_pending_enqueues: producers blocked in put() fail immediately;
  // otherwise they may still complete (TF semantics: close() lets pending
  // enqueues finish unless cancelled).  Consumers drain what is left, then
  // get QueueClosed.
  void close(bool cancel_pending_enqueues) {
    std::lock_guard<std::mutex> lk(mu_);
    closed_ = true;
    cancel_ = cancel_pending_enqueues;
    not_full_.notify_all();
    not_empty_.notify_all();
  }

 private:
  int64_t cap_;
  std::mutex mu_;
  std::condition_variable not_full_, not_empty_;
  std::deque<PyObject*> q_;
  bool closed_ = false, cancel_ = false;
};

void init_queue(py::module& m) {
  py::register_exception<QueueClosed>(m, "QueueClosedError");
  py::register_exception<QueueTimeout>(m, "QueueTimeoutError");
  py::class_<BlockingQueue>(m, "BlockingQueue")
      .def(py::init<int64_t>(), py::arg("capacity"))
      .def_property_readonly("capacity", &BlockingQueue::capacity)
      .def("size", &BlockingQueue::size)
      .def("closed", &BlockingQueue::closed)
      .def("put", &BlockingQueue::put, py::arg("item"), py::arg("timeout") = -1.0)
      .def("put_many", &BlockingQueue::put_many, py::arg("items"), py::arg("timeout") = -1.0)
      .def("get", &BlockingQueue::get, py::arg("timeout") = -1.0)
      .def("get_many", &BlockingQueue::get_many, py::arg("n"), py::arg("timeout") = -1.0,
           py::arg("allow_smaller_final_batch") = false)
      .def("close", &BlockingQueue::close, py::arg("cancel_pending_enqueues") = false);
}

}  // namespace dtf
