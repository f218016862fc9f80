// pybind11 bindings for the native runtime (_native.so).
//
// Exposes: Engine (threaded dependency engine), Var, HostStorage (pooled
// pinned host memory), RecordWriter/RecordReader/RecordPrefetcher, and the
// ImageRecordIter augmenter (AugParam, augment_into, image_resize).
// Python callables pushed to the engine run on worker threads with the GIL
// re-acquired; native tasks (file writes of a bytes buffer) run without it.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdio>
#include <cstring>
#include <memory>

#include "engine.h"
#include "image_aug.h"
#include "recordio.h"
#include "storage.h"

namespace py = pybind11;
using namespace mxamd;

namespace {

struct PyErrorHolder : std::exception {
  explicit PyErrorHolder(py::error_already_set&& e) : err(std::move(e)) {}
  py::error_already_set err;
  const char* what() const noexcept override { return "python exception in engine op"; }
};

void Rethrow(std::exception_ptr p) {
  try {
    std::rethrow_exception(p);
  } catch (PyErrorHolder& h) {
    h.err.restore();
    throw py::error_already_set();
  }
}

}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "mxnet_maintenance_amd native runtime (engine, storage, recordio)";

  py::class_<Var, VarHandle>(m, "Var")
      .def_property_readonly("version", [](const Var& v) { return v.version; })
      .def_property_readonly("name", [](const Var& v) { return v.name; });

  py::class_<Dispatcher>(m, "Dispatcher")
      .def(py::init<bool>(), py::arg("trace") = false)
      .def("set_streams", &Dispatcher::SetStreams, py::arg("device"), py::arg("workers"))
      .def("begin", &Dispatcher::Begin, py::arg("device"), py::arg("cur"), py::arg("reads"))
      .def("write", &Dispatcher::Write, py::arg("device"), py::arg("cur"), py::arg("slot"), py::arg("target"))
      .def("end", &Dispatcher::End, py::arg("device"), py::arg("slot"), py::arg("reads"), py::arg("writes"))
      .def("join", &Dispatcher::Join, py::arg("device"), py::arg("cur"))
      .def_static("slot_of", &Dispatcher::SlotOf)
      .def("take_trace", &Dispatcher::TakeTrace)
      .def_property_readonly("waits", &Dispatcher::waits);

  py::class_<Engine>(m, "Engine")
      .def(py::init<int, bool, bool>(), py::arg("num_workers") = 4, py::arg("naive") = false,
           py::arg("debug") = false)
      .def("new_var", &Engine::NewVar, py::arg("name") = "")
      .def(
          "push",
          [](Engine& e, py::function fn, std::vector<VarHandle> cv, std::vector<VarHandle> mv,
             int priority, std::string name) {
            // The python callable is released with the GIL held right after it
            // runs, so no python reference is dropped on a bare worker thread.
            auto holder = std::make_shared<std::unique_ptr<py::function>>(
                new py::function(std::move(fn)));
            Fn f = [holder]() {
              py::gil_scoped_acquire g;
              try {
                (**holder)();
              } catch (py::error_already_set& err) {
                holder->reset();
                throw PyErrorHolder(std::move(err));
              }
              holder->reset();
            };
            py::gil_scoped_release rel;
            e.Push(std::move(f), cv, mv, priority, name);
          },
          py::arg("fn"), py::arg("const_vars"), py::arg("mutable_vars"), py::arg("priority") = 0,
          py::arg("name") = "")
      .def(
          "push_device",
          [](Engine& e, py::function fn, std::vector<VarHandle> cv, std::vector<VarHandle> mv, uintptr_t stream,
             int device, int priority, std::string name) {
            auto holder = std::make_shared<std::unique_ptr<py::function>>(new py::function(std::move(fn)));
            Fn f = [holder]() {
              py::gil_scoped_acquire g;
              try {
                (**holder)();
              } catch (py::error_already_set& err) {
                holder->reset();
                throw PyErrorHolder(std::move(err));
              }
              holder->reset();
            };
            py::gil_scoped_release rel;
            e.PushDevice(std::move(f), cv, mv, stream, device, priority, name);
          },
          py::arg("fn"), py::arg("const_vars"), py::arg("mutable_vars"), py::arg("stream"), py::arg("device"),
          py::arg("priority") = 0, py::arg("name") = "",
          "Device op: fn enqueues work on `stream`; ordering against other streams is by HIP events.")
      .def("debug_access", &Engine::DebugAccess, py::arg("var"), py::arg("write") = false)
      .def("stream_wait_var",
           [](Engine& e, VarHandle v, uintptr_t stream, int device) {
             try {
               py::gil_scoped_release rel;
               e.StreamWaitVar(v, stream, device);
             } catch (PyErrorHolder&) {
               Rethrow(std::current_exception());
             }
           })
      .def("clear_exception", &Engine::ClearException, py::arg("var"))
      .def_property_readonly("debug", &Engine::debug)
      .def_property_readonly("violations", &Engine::violations)
      .def_property_readonly("last_violation", &Engine::last_violation)
      .def_property_readonly("device_ops", &Engine::device_ops)
      .def(
          "push_write_file",
          [](Engine& e, std::string path, py::bytes data, std::vector<VarHandle> cv,
             std::vector<VarHandle> mv) {
            auto buf = std::make_shared<std::string>(data);
            py::gil_scoped_release rel;
            e.Push(
                [path, buf]() {
                  FILE* fp = std::fopen(path.c_str(), "wb");
                  if (!fp) throw std::runtime_error("cannot open " + path);
                  std::fwrite(buf->data(), 1, buf->size(), fp);
                  std::fclose(fp);
                },
                cv, mv, 0, "write_file");
          },
          "Asynchronously write bytes to a file (no GIL held while writing).")
      .def("wait_for_var",
           [](Engine& e, VarHandle v) {
             try {
               py::gil_scoped_release rel;
               e.WaitForVar(v);
             } catch (PyErrorHolder&) {
               Rethrow(std::current_exception());
             }
           })
      .def("wait_for_all",
           [](Engine& e) {
             try {
               py::gil_scoped_release rel;
               e.WaitForAll();
             } catch (PyErrorHolder&) {
               Rethrow(std::current_exception());
             }
           })
      .def_property_readonly("pending", &Engine::Pending)
      .def_property_readonly("executed", &Engine::executed)
      .def_property_readonly("naive", &Engine::naive)
      .def_property_readonly("num_workers", &Engine::num_workers);

  py::class_<HostStorage>(m, "HostStorage")
      .def(py::init<bool>(), py::arg("pinned") = true)
      .def("alloc", [](HostStorage& s, size_t n) { return reinterpret_cast<uintptr_t>(s.Alloc(n)); })
      .def("free", [](HostStorage& s, uintptr_t p) { s.Free(reinterpret_cast<void*>(p)); })
      .def("release_all", &HostStorage::ReleaseAll)
      .def_property_readonly("pinned", &HostStorage::pinned)
      .def_property_readonly("used_bytes", &HostStorage::used_bytes)
      .def_property_readonly("pooled_bytes", &HostStorage::pooled_bytes)
      .def_property_readonly("hits", &HostStorage::hits)
      .def_property_readonly("misses", &HostStorage::misses)
      .def_static("round_size", &HostStorage::RoundSize);

  py::class_<RecordWriter>(m, "RecordWriter")
      .def(py::init<const std::string&, bool>(), py::arg("path"), py::arg("append") = false)
      .def("write",
           [](RecordWriter& w, py::bytes b) {
             std::string s = b;
             return w.Write(s.data(), s.size());
           })
      .def("tell", &RecordWriter::Tell)
      .def("close", &RecordWriter::Close);

  py::class_<RecordReader>(m, "RecordReader")
      .def(py::init<const std::string&>())
      .def("read",
           [](RecordReader& r) -> py::object {
             std::string s;
             bool ok;
             {
               py::gil_scoped_release rel;
               ok = r.Next(&s);
             }
             if (!ok) return py::none();
             return py::bytes(s);
           })
      .def("seek", &RecordReader::Seek)
      .def("tell", &RecordReader::Tell)
      .def("close", &RecordReader::Close);

  py::class_<RecordPrefetcher>(m, "RecordPrefetcher")
      .def(py::init<const std::string&, std::vector<uint64_t>, size_t>())
      .def("next", [](RecordPrefetcher& p) -> py::object {
        std::string s;
        bool ok;
        {
          py::gil_scoped_release rel;
          ok = p.Next(&s);
        }
        if (!ok) return py::none();
        return py::bytes(s);
      });
  py::class_<AugParam>(m, "AugParam")
      .def(py::init<>())
      .def_readwrite("out_c", &AugParam::out_c)
      .def_readwrite("out_h", &AugParam::out_h)
      .def_readwrite("out_w", &AugParam::out_w)
      .def_readwrite("resize", &AugParam::resize)
      .def_readwrite("rand_crop", &AugParam::rand_crop)
      .def_readwrite("random_resized_crop", &AugParam::random_resized_crop)
      .def_readwrite("max_rotate_angle", &AugParam::max_rotate_angle)
      .def_readwrite("max_aspect_ratio", &AugParam::max_aspect_ratio)
      .def_readwrite("has_min_aspect_ratio", &AugParam::has_min_aspect_ratio)
      .def_readwrite("min_aspect_ratio", &AugParam::min_aspect_ratio)
      .def_readwrite("max_shear_ratio", &AugParam::max_shear_ratio)
      .def_readwrite("max_crop_size", &AugParam::max_crop_size)
      .def_readwrite("min_crop_size", &AugParam::min_crop_size)
      .def_readwrite("max_random_scale", &AugParam::max_random_scale)
      .def_readwrite("min_random_scale", &AugParam::min_random_scale)
      .def_readwrite("max_random_area", &AugParam::max_random_area)
      .def_readwrite("min_random_area", &AugParam::min_random_area)
      .def_readwrite("min_img_size", &AugParam::min_img_size)
      .def_readwrite("max_img_size", &AugParam::max_img_size)
      .def_readwrite("brightness", &AugParam::brightness)
      .def_readwrite("contrast", &AugParam::contrast)
      .def_readwrite("saturation", &AugParam::saturation)
      .def_readwrite("pca_noise", &AugParam::pca_noise)
      .def_readwrite("random_h", &AugParam::random_h)
      .def_readwrite("random_s", &AugParam::random_s)
      .def_readwrite("random_l", &AugParam::random_l)
      .def_readwrite("rotate", &AugParam::rotate)
      .def_readwrite("rotate_list", &AugParam::rotate_list)
      .def_readwrite("fill_value", &AugParam::fill_value)
      .def_readwrite("inter_method", &AugParam::inter_method)
      .def_readwrite("pad", &AugParam::pad)
      .def_readwrite("mirror", &AugParam::mirror)
      .def_readwrite("rand_mirror", &AugParam::rand_mirror)
      .def_readwrite("scale", &AugParam::scale)
      .def_readwrite("max_random_contrast", &AugParam::max_random_contrast)
      .def_readwrite("max_random_illumination", &AugParam::max_random_illumination)
      .def_readwrite("mean_img", &AugParam::mean_img)
      .def_property(
          "mean", [](const AugParam& p) { return std::vector<float>(p.mean, p.mean + 4); },
          [](AugParam& p, const std::vector<float>& v) {
            for (size_t i = 0; i < 4 && i < v.size(); ++i) p.mean[i] = v[i];
          })
      .def_property(
          "std", [](const AugParam& p) { return std::vector<float>(p.std_, p.std_ + 4); },
          [](AugParam& p, const std::vector<float>& v) {
            for (size_t i = 0; i < 4 && i < v.size(); ++i) p.std_[i] = v[i];
          })
      .def("check", &CheckAugParam);

  // Augment one decoded HWC uint8 image and write it, normalised, into `out`
  // (a batch slot of data_shape in CHW or HWC order; float32, uint8 or int8).
  // Runs without the GIL.  Raises ValueError on invalid input.
  m.def(
      "augment_into",
      [](py::array_t<uint8_t, py::array::c_style | py::array::forcecast> img, const AugParam& p,
         uint32_t seed, py::array out, bool nchw) {
        if (img.ndim() != 3 && img.ndim() != 2) throw py::value_error("image must be HxW or HxWxC uint8");
        Image src(int(img.shape(0)), int(img.shape(1)), img.ndim() == 3 ? int(img.shape(2)) : 1);
        if (src.c != 1 && src.c != 3 && src.c != 4) throw py::value_error("image must have 1, 3 or 4 channels");
        std::memcpy(src.px.data(), img.data(), src.px.size());
        OutType t;
        if (out.dtype().is(py::dtype::of<float>()))
          t = OutType::kFloat32;
        else if (out.dtype().is(py::dtype::of<uint8_t>()))
          t = OutType::kUint8;
        else if (out.dtype().is(py::dtype::of<int8_t>()))
          t = OutType::kInt8;
        else
          throw py::value_error("augment_into: output must be float32, uint8 or int8");
        if (!(out.flags() & py::array::c_style) || !out.writeable())
          throw py::value_error("augment_into: output must be a writable C-contiguous array");
        if (size_t(out.size()) != size_t(p.out_c) * p.out_h * p.out_w)
          throw py::value_error("augment_into: output size does not match data_shape");
        void* dst = out.mutable_data();
        std::string err;
        {
          py::gil_scoped_release rel;
          try {
            std::mt19937 rng(seed);
            Image res = Augment(src, p, rng);
            WriteNormalized(res, p, rng, dst, t, nchw);
          } catch (const std::exception& e) {
            err = e.what();
          }
        }
        if (!err.empty()) throw py::value_error(err);
      },
      py::arg("img"), py::arg("param"), py::arg("seed"), py::arg("out"), py::arg("nchw") = true);

  m.def(
      "image_resize",
      [](py::array_t<uint8_t, py::array::c_style | py::array::forcecast> img, int w, int h, int inter) {
        if (img.ndim() != 3) throw py::value_error("image must be HxWxC uint8");
        Image src(int(img.shape(0)), int(img.shape(1)), int(img.shape(2)));
        std::memcpy(src.px.data(), img.data(), src.px.size());
        Image d;
        {
          py::gil_scoped_release rel;
          d = Resize(src, w, h, inter);
        }
        py::array_t<uint8_t> out({d.h, d.w, d.c});
        std::memcpy(out.mutable_data(), d.px.data(), d.px.size());
        return out;
      },
      py::arg("img"), py::arg("w"), py::arg("h"), py::arg("inter") = 1);
}
