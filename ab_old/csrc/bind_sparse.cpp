// The one-GPU sparse logistic-regression step of lr2.py as ONE host call
// (csrc/kernels/sparse_lr.hip).  SparseLRPlan.run takes lr2.py's own feed
// arrays -- labels y [B, 1], SparseTensor indices [nnz, 2] (row, column),
// feature ids [nnz], values [nnz] (lr2.py:440-446) -- builds the CSR row
// offsets (a stable counting sort when the COO entries are not in row order),
// packs ids | offsets | values | labels into a pinned staging slot (mapped,
// coherent host memory) with the GIL released and issues the two step kernels
// on the caller's stream: the forward kernel reads the slot in place and leaves
// device copies of ids / offsets / values for the apply kernel (DTF_SLR_FEED=
// stage: a staging kernel copies the slot first; =dma: an SDMA hipMemcpyAsync,
// which ran as a 36 us blit and cost ~40 us of host time per call on MI355X --
// profiles/lr2_compat_r5.json).  Returns without waiting (staging slots are
// double buffered behind events).  SparseLRPlan.step runs the same kernels on device
// tensors (models/sparse_lr.py, one worker).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <pybind11/numpy.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

extern "C" {
hipError_t dtfk_slr_step(float* W, long long F, const void* ids, int ids32, const long long* offsets,
                         const float* vals, const float* labels, float* bias, int B, const float* lr_ptr, float lr_val,
                         float* dz, float* lrow, float* loss_out, int* bad, void* gvar, int gkind, hipStream_t stream);
hipError_t dtfk_slr_stage(const void* src, void* dst, long long bytes, hipStream_t stream);
void dtfk_slr_set_rows_per_wg(int rpw);
hipError_t dtfk_slr_step_direct(float* W, long long F, const void* hids, int ids32, const long long* hoffsets,
                                const float* hvals, const float* hlabels, void* ids_d, long long* off_d, float* vals_d,
                                float* bias, int B, float lr_val, float* dz, float* lrow, float* loss_out, int* bad,
                                void* gvar, int gkind, hipStream_t stream);
}

namespace dtf {

static void hck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

static int64_t align16(int64_t v) { return (v + 15) / 16 * 16; }

class SparseLRPlan {
 public:
  SparseLRPlan(at::Tensor W, at::Tensor bias, c10::optional<at::Tensor> gstep) : W_(W), bias_(bias) {
    TORCH_CHECK(W.is_cuda() && W.scalar_type() == at::kFloat && W.is_contiguous() &&
                    (W.dim() == 1 || (W.dim() == 2 && W.size(1) == 1)),
                "SparseLRPlan: W must be a contiguous fp32 [F, 1] GPU table");
    TORCH_CHECK(bias.is_cuda() && bias.scalar_type() == at::kFloat && bias.numel() == 1 && bias.is_contiguous(),
                "SparseLRPlan: bias must be one fp32 GPU value");
    F_ = W.size(0);
    if (gstep.has_value()) {
      const at::Tensor& g = *gstep;
      TORCH_CHECK(g.is_cuda() && g.numel() == 1, "SparseLRPlan: device scalar global_step");
      switch (g.scalar_type()) {
        case at::kFloat: gkind_ = 1; break;
        case at::kLong: gkind_ = 2; break;
        case at::kInt: gkind_ = 3; break;
        case at::kDouble: gkind_ = 4; break;
        default: TORCH_CHECK(false, "SparseLRPlan: unsupported global_step dtype");
      }
      gstep_ = g;
    }
    auto fo = W.options();
    loss_ = at::zeros({1}, fo);
    bad_ = at::zeros({1}, fo.dtype(at::kInt));
    for (int i = 0; i < 2; ++i) hck(hipEventCreateWithFlags(&ev_[i], hipEventDisableTiming), "hipEventCreate");
    const char* fe = std::getenv("DTF_SLR_FEED");
    const std::string f = fe != nullptr ? fe : "direct";
    feed_ = f == "dma" ? 2 : (f == "stage" ? 1 : (f == "overlap" ? 3 : 0));
    const char* rp = std::getenv("DTF_SLR_RPW");
    dtfk_slr_set_rows_per_wg(rp != nullptr ? std::atoi(rp) : 32);
    if (feed_ == 3) {
      // the next batch's staging copy runs on a queue of its own, under the
      // current step's kernels (a CU mask is a queue property: a CU-masked stream
      // does not share a hardware queue with the compute stream)
      int ncu = 0;
      (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, W.get_device());
      std::vector<uint32_t> mask((size_t)std::max(1, (ncu + 31) / 32), 0xffffffffu);
      if (ncu <= 0 || hipExtStreamCreateWithCUMask(&side_, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
        (void)hipGetLastError();
        hck(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking), "SparseLRPlan: side stream");
      }
      for (int i = 0; i < 2; ++i) hck(hipEventCreateWithFlags(&evs_[i], hipEventDisableTiming), "hipEventCreate");
    }
  }
  ~SparseLRPlan() {
    for (int i = 0; i < 2; ++i) {
      if (pending_[i]) (void)hipEventSynchronize(ev_[i]);
      if (ev_[i]) (void)hipEventDestroy(ev_[i]);
      if (hbuf_[i]) (void)hipHostFree(hbuf_[i]);
      if (evs_[i]) (void)hipEventDestroy(evs_[i]);
    }
    if (side_) (void)hipStreamDestroy(side_);
  }

  // lr2.py's feeds (numpy).  False: not applicable (dtypes, shapes, a row index
  // outside [0, B)) -- nothing ran, the caller takes the general path.
  bool run(py::array y, py::array idx, py::array ids, py::array vals, double lr) {
    if (!y.dtype().is(py::dtype::of<float>()) || !idx.dtype().is(py::dtype::of<int64_t>()) ||
        !ids.dtype().is(py::dtype::of<int64_t>()) || !vals.dtype().is(py::dtype::of<float>()))
      return false;
    const int64_t B = y.size(), n = ids.size();
    if (B < 1 || B > (1 << 30) || vals.size() != n || (n > 0 && (idx.ndim() != 2 || idx.shape(0) != n || idx.shape(1) < 2)))
      return false;
    // strided views are fine: read through the numpy strides
    const char* yb = static_cast<const char*>(y.data());
    const char* ib = static_cast<const char*>(idx.data());
    const char* fb = static_cast<const char*>(ids.data());
    const char* vb = static_cast<const char*>(vals.data());
    const int64_t ys = y.ndim() >= 1 ? y.strides(0) : 4;
    const int64_t is0 = n > 0 ? idx.strides(0) : 0;
    const int64_t fs = ids.ndim() >= 1 ? ids.strides(0) : 8, vs = vals.ndim() >= 1 ? vals.strides(0) : 4;
    if (y.ndim() > 2 || ids.ndim() > 1 || vals.ndim() > 1 || (y.ndim() == 2 && y.shape(1) != 1 && y.shape(0) != 1))
      return false;
    const int64_t ys_el = (y.ndim() == 2 && y.shape(0) == 1) ? y.strides(1) : ys;
    return submit_(B, n, lr, [&](int64_t* hoff, int64_t* hid, int32_t* hid32, float* hval, float* hlab, bool i32) {
      // rows -> CSR offsets: in row order (lr2.py's own feeds, as_tf_feed) the
      // offsets are the row boundaries, found in one pass; otherwise a stable
      // counting sort by row (the same bags: the 'sum' combiner)
      bool ok = true, sorted = true;
      auto row = [&](int64_t j) { return *reinterpret_cast<const int64_t*>(ib + j * is0); };
      // one pass: row range, order and (in order) the CSR boundaries -- the
      // common case, lr2.py's own row-major feeds (as_tf_feed); a row out of
      // order sends the batch to the stable counting sort below
      int64_t prev = n > 0 ? row(0) : B;
      if (n > 0 && (prev < 0 || prev >= B)) return false;
      for (int64_t b = 0; b <= prev && b <= B; ++b) hoff[b] = 0;
      for (int64_t j = 1; j < n; ++j) {
        const int64_t r = row(j);
        if (r != prev) {
          if (r < prev || r >= B) {
            sorted = false;
            break;
          }
          for (int64_t b = prev + 1; b <= r; ++b) hoff[b] = j;
          prev = r;
        }
      }
      if (sorted) {
        for (int64_t b = prev + 1; b <= B; ++b) hoff[b] = n;
      } else {
        for (int64_t j = 0; j < n && ok; ++j) {
          const int64_t r = row(j);
          ok = r >= 0 && r < B;
        }
      }
      if (!ok) return false;
      if (sorted) {
        pack_ids_(hid, hid32, i32, fb, fs, n);
        if (vs == 4) std::memcpy(hval, vb, 4 * (size_t)n);
        else for (int64_t j = 0; j < n; ++j) hval[j] = *reinterpret_cast<const float*>(vb + j * vs);
      } else {
        std::vector<int64_t>& cnt = cnt_;
        cnt.assign((size_t)B + 1, 0);
        for (int64_t j = 0; j < n; ++j) ++cnt[(size_t)row(j) + 1];
        for (int64_t b = 0; b < B; ++b) cnt[(size_t)b + 1] += cnt[(size_t)b];
        std::memcpy(hoff, cnt.data(), sizeof(int64_t) * (size_t)(B + 1));
        const int64_t F = F_;
        for (int64_t j = 0; j < n; ++j) {
          const int64_t dd = cnt[(size_t)row(j)]++;
          const int64_t id = *reinterpret_cast<const int64_t*>(fb + j * fs);
          if (i32) hid32[dd] = ((uint64_t)id < (uint64_t)F) ? (int32_t)id : -1;
          else hid[dd] = id;
          hval[dd] = *reinterpret_cast<const float*>(vb + j * vs);
        }
      }
      for (int64_t b = 0; b < B; ++b) hlab[b] = *reinterpret_cast<const float*>(yb + b * ys_el);
      return true;
    });
  }

  // A host CSR batch (the native trainer's own layout: labels [B] / [B, 1] f32,
  // offsets [B + 1] i64, ids [nnz] i64, vals [nnz] f32 or None) through the same
  // packed feed.  False: not applicable (dtypes / shapes / offsets not a CSR of nnz).
  bool run_csr(py::array y, py::array offsets, py::array ids, py::object vals_o, double lr) {
    if (!y.dtype().is(py::dtype::of<float>()) || !offsets.dtype().is(py::dtype::of<int64_t>()) ||
        !ids.dtype().is(py::dtype::of<int64_t>()))
      return false;
    py::array vals;
    const bool has_v = !vals_o.is_none();
    if (has_v) {
      vals = py::array::ensure(vals_o);
      if (!vals || !vals.dtype().is(py::dtype::of<float>()) || vals.ndim() != 1 || vals.size() != ids.size()) return false;
    }
    const int64_t B = y.size(), n = ids.size();
    if (B < 1 || B > (1 << 30) || offsets.ndim() != 1 || offsets.size() != B + 1 || ids.ndim() != 1) return false;
    const char* yb = static_cast<const char*>(y.data());
    const char* ob = static_cast<const char*>(offsets.data());
    const char* fb = static_cast<const char*>(ids.data());
    const char* vb = has_v ? static_cast<const char*>(vals.data()) : nullptr;
    const int64_t ys = (y.ndim() == 2 && y.shape(0) == 1) ? y.strides(1) : (y.ndim() >= 1 ? y.strides(0) : 4);
    const int64_t os = offsets.strides(0), fs = ids.strides(0), vs = has_v ? vals.strides(0) : 4;
    if (y.ndim() > 2 || (y.ndim() == 2 && y.shape(1) != 1 && y.shape(0) != 1)) return false;
    return submit_(B, n, lr, [&](int64_t* hoff, int64_t* hid, int32_t* hid32, float* hval, float* hlab, bool i32) {
      int64_t prev = 0;
      for (int64_t b = 0; b <= B; ++b) {
        const int64_t o = *reinterpret_cast<const int64_t*>(ob + b * os);
        if (o < prev || o > n || (b == 0 && o != 0)) return false;
        hoff[b] = prev = o;
      }
      if (hoff[B] != n) return false;
      pack_ids_(hid, hid32, i32, fb, fs, n);
      if (!has_v) for (int64_t j = 0; j < n; ++j) hval[j] = 1.f;
      else if (vs == 4) std::memcpy(hval, vb, 4 * (size_t)n);
      else for (int64_t j = 0; j < n; ++j) hval[j] = *reinterpret_cast<const float*>(vb + j * vs);
      for (int64_t b = 0; b < B; ++b) hlab[b] = *reinterpret_cast<const float*>(yb + b * ys);
      return true;
    });
  }

 private:
  // out-of-range ids are kept as such (the kernels count and skip them): in
  // int32 form anything outside [0, F) becomes -1
  void pack_ids_(int64_t* hid, int32_t* hid32, bool i32, const char* fb, int64_t fs, int64_t n) const {
    const int64_t F = F_;
    if (i32 && fs == 8) {
      const int64_t* f = reinterpret_cast<const int64_t*>(fb);
      for (int64_t j = 0; j < n; ++j) hid32[j] = ((uint64_t)f[j] < (uint64_t)F) ? (int32_t)f[j] : -1;
    } else if (!i32 && fs == 8) {
      std::memcpy(hid, fb, 8 * (size_t)n);
    } else {
      for (int64_t j = 0; j < n; ++j) {
        const int64_t id = *reinterpret_cast<const int64_t*>(fb + j * fs);
        if (i32) hid32[j] = ((uint64_t)id < (uint64_t)F) ? (int32_t)id : -1;
        else hid[j] = id;
      }
    }
  }

  // Packs one batch (fill writes the CSR offsets, ids, values and labels into
  // the pinned slot) with the GIL released, moves it to the device and launches
  // the step.  False when fill refused the batch (nothing was launched).
  template <typename Fill>
  bool submit_(int64_t B, int64_t n, double lr, Fill&& fill) {
    // ids travel as int32 when the table has < 2^31 rows (lr2's F = 1e9 does): half the bytes
    const bool i32 = F_ < (1LL << 31);
    const int64_t isz = i32 ? 4 : 8;
    const int64_t o_ids = 0, o_off = align16(isz * n), o_val = o_off + align16(8 * (B + 1)),
                  o_lab = o_val + align16(4 * n), total = o_lab + align16(4 * B);
    const int slot = slot_ ^ 1;
    bool ok = true;
    if (dz_.numel() < B) {
      dz_ = at::empty({std::max<int64_t>(B, 1024)}, W_.options());
      lrow_ = at::empty({std::max<int64_t>(B, 1024)}, W_.options());
    }
    at::Tensor& dvb = feed_ == 3 ? dev2_[slot] : dev_;   // overlap: one device copy per slot
    if (dvb.numel() < total) dvb = at::empty({std::max<int64_t>(total, 1 << 20)}, W_.options().dtype(at::kByte));
    hipStream_t st = c10::hip::getCurrentHIPStream().stream();
    char* d = static_cast<char*>(dvb.data_ptr());
    {
      py::gil_scoped_release nogil;
      using clk = std::chrono::steady_clock;
      const auto t0 = clk::now();
      if (pending_[slot]) hck(hipEventSynchronize(ev_[slot]), "SparseLRPlan: staging slot");
      pending_[slot] = false;
      if (hcap_[slot] < total) {   // mapped + coherent: the staging kernel reads it in place
        if (hbuf_[slot]) hck(hipHostFree(hbuf_[slot]), "hipHostFree");
        hbuf_[slot] = nullptr;
        const int64_t cap = std::max<int64_t>(total, 1 << 20);
        hck(hipHostMalloc(&hbuf_[slot], (size_t)cap, hipHostMallocMapped | hipHostMallocCoherent),
            "SparseLRPlan: pinned staging slot");
        hck(hipHostGetDevicePointer(&hdev_[slot], hbuf_[slot], 0), "SparseLRPlan: staging slot device view");
        hcap_[slot] = cap;
      }
      const auto tw = clk::now();   // slot wait (+ first-use allocation) | packing
      char* h = static_cast<char*>(hbuf_[slot]);
      ok = fill(reinterpret_cast<int64_t*>(h + o_off), reinterpret_cast<int64_t*>(h + o_ids),
                reinterpret_cast<int32_t*>(h + o_ids), reinterpret_cast<float*>(h + o_val),
                reinterpret_cast<float*>(h + o_lab), i32);
      if (ok) {
        slot_ = slot;
        const auto t1 = clk::now();
        if (feed_ == 0) {
          // the forward kernel reads the slot in place and leaves device copies for the apply
          const char* hd = static_cast<const char*>(hdev_[slot]);
          hck(dtfk_slr_step_direct(W_.data_ptr<float>(), (long long)F_, hd + o_ids, i32 ? 1 : 0,
                                   reinterpret_cast<const long long*>(hd + o_off),
                                   reinterpret_cast<const float*>(hd + o_val), reinterpret_cast<const float*>(hd + o_lab),
                                   d + o_ids, reinterpret_cast<long long*>(d + o_off), reinterpret_cast<float*>(d + o_val),
                                   bias_.data_ptr<float>(), (int)B, (float)lr, dz_.data_ptr<float>(),
                                   lrow_.data_ptr<float>(), loss_.data_ptr<float>(), bad_.data_ptr<int>(),
                                   gkind_ ? gstep_.data_ptr() : nullptr, gkind_, st),
              "SparseLRPlan: step");
          hck(hipEventRecord(ev_[slot], st), "SparseLRPlan: event");
          pending_[slot] = true;
        } else if (feed_ == 3) {
          hck(dtfk_slr_stage(hdev_[slot], d, total, side_), "SparseLRPlan: feed staging");
          hck(hipEventRecord(evs_[slot], side_), "SparseLRPlan: event");
          hck(hipStreamWaitEvent(st, evs_[slot], 0), "SparseLRPlan: wait staging");
          launch(d + o_ids, i32, reinterpret_cast<const long long*>(d + o_off), reinterpret_cast<const float*>(d + o_val),
                 reinterpret_cast<const float*>(d + o_lab), (int)B, (float)lr, st);
          hck(hipEventRecord(ev_[slot], st), "SparseLRPlan: event");   // host + device slot free after the step
          pending_[slot] = true;
        } else {
          if (feed_ == 2) hck(hipMemcpyAsync(d, h, (size_t)total, hipMemcpyHostToDevice, st), "SparseLRPlan: feed copy");
          else hck(dtfk_slr_stage(hdev_[slot], d, total, st), "SparseLRPlan: feed staging");
          hck(hipEventRecord(ev_[slot], st), "SparseLRPlan: event");
          pending_[slot] = true;
          launch(d + o_ids, i32, reinterpret_cast<const long long*>(d + o_off), reinterpret_cast<const float*>(d + o_val),
                 reinterpret_cast<const float*>(d + o_lab), (int)B, (float)lr, st);
        }
        t_[2] += std::chrono::duration<double, std::micro>(tw - t0).count();
        t_[0] += std::chrono::duration<double, std::micro>(t1 - tw).count();
        t_[1] += std::chrono::duration<double, std::micro>(clk::now() - t1).count();
      }
    }
    if (!ok) return false;
    ++runs_;
    return true;
  }

 public:
  // device tensors (labels [B] / [B,1] f32, offsets [B+1] i64, ids [nnz] i64, vals [nnz] f32 or None)
  at::Tensor step(at::Tensor labels, at::Tensor offsets, at::Tensor ids, c10::optional<at::Tensor> vals, double lr) {
    TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kFloat && labels.is_contiguous(), "labels");
    TORCH_CHECK(offsets.is_cuda() && offsets.scalar_type() == at::kLong && offsets.is_contiguous(), "offsets");
    TORCH_CHECK(ids.is_cuda() && ids.scalar_type() == at::kLong && ids.is_contiguous(), "ids");
    const int64_t B = labels.numel();
    TORCH_CHECK(offsets.numel() == B + 1, "SparseLRPlan.step: offsets must hold B + 1 entries");
    const float* vp = nullptr;
    if (vals.has_value()) {
      TORCH_CHECK(vals->is_cuda() && vals->scalar_type() == at::kFloat && vals->is_contiguous() &&
                      vals->numel() == ids.numel(), "vals");
      vp = vals->data_ptr<float>();
    }
    if (dz_.numel() < B) {
      dz_ = at::empty({std::max<int64_t>(B, 1024)}, W_.options());
      lrow_ = at::empty({std::max<int64_t>(B, 1024)}, W_.options());
    }
    launch(ids.data_ptr(), false, reinterpret_cast<const long long*>(offsets.data_ptr<int64_t>()), vp,
           labels.data_ptr<float>(), (int)B, (float)lr, c10::hip::getCurrentHIPStream().stream());
    ++runs_;
    return loss();
  }

  at::Tensor loss() const { return loss_.select(0, 0); }   // the last run's mean loss (0-d, device)
  // host time per run() call, us: waiting for the staging slot (the GPU two
  // steps behind), feed packing (CSR build + copies into the pinned slot), then
  // the feed transfer + two launches
  py::dict timing() const {
    py::dict dd;
    const double k = runs_ > 0 ? (double)runs_ : 1.0;
    dd["pack_us"] = t_[0] / k;
    dd["enqueue_us"] = t_[1] / k;
    dd["slot_wait_us"] = t_[2] / k;
    dd["runs"] = runs_;
    dd["feed"] = feed_ == 2 ? "dma" : (feed_ == 1 ? "staging kernel" : (feed_ == 3 ? "overlapped staging" : "direct"));
    return dd;
  }
  int64_t runs() const { return runs_; }
  int64_t bad_ids() const { return bad_.item<int>(); }

 private:
  void launch(const void* ids, bool i32, const long long* offs, const float* vals, const float* labels, int B,
              float lr, hipStream_t st) {
    hck(dtfk_slr_step(W_.data_ptr<float>(), (long long)F_, ids, i32 ? 1 : 0, offs, vals, labels, bias_.data_ptr<float>(), B, nullptr,
                      lr, dz_.data_ptr<float>(), lrow_.data_ptr<float>(), loss_.data_ptr<float>(),
                      bad_.data_ptr<int>(), gkind_ ? gstep_.data_ptr() : nullptr, gkind_, st),
        "SparseLRPlan: step");
  }

  at::Tensor W_, bias_, gstep_, loss_, bad_, dev_, dz_, lrow_;
  void* hbuf_[2] = {nullptr, nullptr};
  void* hdev_[2] = {nullptr, nullptr};
  int64_t hcap_[2] = {0, 0};
  int feed_ = 0;   // 0 direct (the forward reads the pinned slot), 1 staging kernel, 2 SDMA copy, 3 staging on a side queue
  hipStream_t side_ = nullptr;
  hipEvent_t evs_[2] = {nullptr, nullptr};
  at::Tensor dev2_[2];
  std::vector<int64_t> cnt_;
  hipEvent_t ev_[2] = {nullptr, nullptr};
  bool pending_[2] = {false, false};
  int slot_ = 0, gkind_ = 0;
  int64_t F_ = 0, runs_ = 0;
  double t_[3] = {0, 0, 0};
};

void init_sparse(py::module& m) {
  py::class_<SparseLRPlan>(m, "SparseLRPlan")
      .def(py::init<at::Tensor, at::Tensor, c10::optional<at::Tensor>>(), py::arg("W"), py::arg("bias"),
           py::arg("gstep") = py::none())
      .def("run", &SparseLRPlan::run, py::arg("y"), py::arg("indices"), py::arg("ids"), py::arg("vals"), py::arg("lr"))
      .def("run_csr", &SparseLRPlan::run_csr, py::arg("y"), py::arg("offsets"), py::arg("ids"), py::arg("vals"),
           py::arg("lr"))
      .def("step", &SparseLRPlan::step, py::arg("labels"), py::arg("offsets"), py::arg("ids"), py::arg("vals"),
           py::arg("lr"))
      .def("loss", &SparseLRPlan::loss)
      .def("runs", &SparseLRPlan::runs)
      .def("timing", &SparseLRPlan::timing)
      .def("bad_ids", &SparseLRPlan::bad_ids);
}

}  // namespace dtf
