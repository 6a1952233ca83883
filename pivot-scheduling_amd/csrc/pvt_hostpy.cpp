// pvt_hostpy.cpp — the lock-step driver's host-side marshalling in C++ (a CPython extension,
// pivot_place._hostbatch). PlacementEngine.place_host_batch hands it the rounds of one tick as
// (RoundArrays, cost_aware items or None) pairs; it fills the pvt_round / pvt_ca_items
// descriptors straight from the numpy buffers, allocates the result arrays, and calls
// pvt_place_host_batch (include/pivot_place.h) through the function pointer the ctypes binding
// resolved -- one C++ pass per tick instead of ~25 us of ctypes attribute traffic per round.
// Nothing here computes a placement: the engine (libpivot_place.so) does, on the GPU.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <cstring>
#include <stdexcept>
#include <vector>

#include "pivot_place.h"

namespace py = pybind11;

namespace {

using batch_fn = int (*)(pvt_ctx*, pvt_round*, pvt_ca_items* const*, int32_t, int32_t*);

template <class T>
using carr = py::array_t<T, py::array::c_style | py::array::forcecast>;

// A C-contiguous array of T over `o` (no copy when it already is one), kept alive in `keep`.
template <class T>
const T* data_of(py::handle o, std::vector<py::object>& keep) {
  if (o.is_none()) return nullptr;
  carr<T> a = carr<T>::ensure(o);
  if (!a) throw std::runtime_error("pivot_place._hostbatch: array conversion failed");
  keep.push_back(a);
  return a.data();
}

}  // namespace

// place_host_batch(fn, ctx, rounds, items) -> (results, rcs)
//   rounds: RoundArrays objects; items: per round None or the tuple (task_item, pred_off,
//   pred_host, item_app, n_apps, storage_zone, zone_storage, mt_state).
//   results[i] = (placement, order, avail, mt_state or None, items_mt or None, status or None)
static py::tuple place_host_batch(std::uintptr_t fn, std::uintptr_t ctx, py::list rounds, py::list items) {
  const size_t n = rounds.size();
  if (items.size() != n) throw std::invalid_argument("rounds and items differ in length");
  std::vector<pvt_round> rs(n);
  std::vector<pvt_ca_items> its(n);
  std::vector<pvt_ca_items*> itp(n, nullptr);
  std::vector<int32_t> rcs(n, 0);
  std::vector<py::object> keep;
  keep.reserve(n * 12);
  py::list results;
  for (size_t i = 0; i < n; i++) {
    py::handle r = rounds[i];
    pvt_round& s = rs[i];
    std::memset(&s, 0, sizeof(s));
    carr<double> av_in = carr<double>::ensure(r.attr("avail"));
    carr<double> dem = carr<double>::ensure(r.attr("dem"));
    carr<double> cost = carr<double>::ensure(r.attr("cost"));
    if (!av_in || !dem || !cost || av_in.ndim() != 2 || dem.ndim() != 2 || cost.ndim() != 2 ||
        av_in.shape(0) != 4 || dem.shape(0) != 4)
      throw std::invalid_argument("round arrays of the wrong shape");
    const int H = (int)av_in.shape(1), T = (int)dem.shape(1);
    keep.push_back(dem);
    keep.push_back(cost);
    s.mode = r.attr("mode").cast<int>();
    s.n_hosts = H;
    s.n_tasks = T;
    s.n_zones = (int)cost.shape(0);
    py::object ga = r.attr("group_anchor");
    s.n_groups = ga.is_none() ? 0 : (int)py::len(ga);
    s.sort_tasks = r.attr("sort_tasks").cast<bool>() ? 1 : 0;
    s.sort_hosts = r.attr("sort_hosts").cast<bool>() ? 1 : 0;
    py::array_t<double> avail({(py::ssize_t)4, (py::ssize_t)H});
    std::memcpy(avail.mutable_data(), av_in.data(), sizeof(double) * 4 * (size_t)H);
    py::array_t<int32_t> placement((py::ssize_t)T), order((py::ssize_t)T);
    s.avail = avail.mutable_data();
    s.placement = placement.mutable_data();
    s.order = order.mutable_data();
    s.dem = dem.data();
    s.cost = cost.data();
    s.zone = data_of<int32_t>(r.attr("zone"), keep);
    s.bw = data_of<double>(r.attr("bw"), keep);
    s.tiebreak = data_of<uint32_t>(r.attr("tiebreak"), keep);
    s.decay = data_of<int32_t>(r.attr("decay"), keep);
    s.task_group = data_of<int32_t>(r.attr("task_group"), keep);
    s.group_anchor = data_of<int32_t>(ga, keep);
    s.rt_bw = data_of<double>(r.attr("rt_bw"), keep);
    py::object mt = py::none();
    py::object mt_in = r.attr("mt_state");
    if (!mt_in.is_none()) {
      carr<uint32_t> m0 = carr<uint32_t>::ensure(mt_in);
      if (!m0 || m0.size() != 625) throw std::invalid_argument("mt_state must hold 625 words");
      py::array_t<uint32_t> m((py::ssize_t)625);
      std::memcpy(m.mutable_data(), m0.data(), sizeof(uint32_t) * 625);
      s.mt_state = m.mutable_data();
      mt = m;
    }
    py::object imt = py::none(), st = py::none();
    py::handle ca = items[i];
    if (!ca.is_none()) {
      py::tuple c = py::reinterpret_borrow<py::tuple>(ca);
      pvt_ca_items& it = its[i];
      std::memset(&it, 0, sizeof(it));
      carr<int32_t> ti = carr<int32_t>::ensure(c[0]);
      carr<int64_t> off = carr<int64_t>::ensure(c[1]);
      carr<int32_t> ph = carr<int32_t>::ensure(c[2]);
      carr<int32_t> ia = carr<int32_t>::ensure(c[3]);
      carr<int32_t> sz = carr<int32_t>::ensure(c[5]);
      carr<int32_t> zs = carr<int32_t>::ensure(c[6]);
      carr<uint32_t> m0 = carr<uint32_t>::ensure(c[7]);
      if (!ti || !off || !ph || !ia || !sz || !zs || !m0) throw std::invalid_argument("bad items");
      if (m0.size() != 625) throw std::invalid_argument("items mt_state must hold 625 words");
      for (py::object o : {py::object(ti), py::object(off), py::object(ph), py::object(ia),
                           py::object(sz), py::object(zs)})
        keep.push_back(o);
      py::array_t<uint32_t> m((py::ssize_t)625);
      std::memcpy(m.mutable_data(), m0.data(), sizeof(uint32_t) * 625);
      py::array_t<int32_t> status((py::ssize_t)2);
      status.mutable_data()[0] = status.mutable_data()[1] = 0;
      it.n_items = (int32_t)ia.size();
      it.n_apps = c[4].cast<int32_t>();
      it.n_pred = (int64_t)ph.size();
      it.task_item = ti.data();
      it.pred_off = off.data();
      it.pred_host = ph.data();
      it.item_app = ia.data();
      it.n_storage = (int32_t)sz.size();
      it.reserved = 0;
      it.storage_zone = sz.data();
      it.zone_storage = zs.data();
      it.mt_state = m.mutable_data();
      it.status = status.mutable_data();
      itp[i] = &it;
      imt = m;
      st = status;
    }
    results.append(py::make_tuple(placement, order, avail, mt, imt, st));
  }
  int rc;
  {
    py::gil_scoped_release nogil;     // (the simulation threads may run while the GPU works)
    rc = reinterpret_cast<batch_fn>(fn)(reinterpret_cast<pvt_ctx*>(ctx), rs.data(), itp.data(),
                                        (int32_t)n, rcs.data());
  }
  py::list rl;
  for (size_t i = 0; i < n; i++) rl.append(rcs[i]);
  return py::make_tuple(rc, results, rl);
}

PYBIND11_MODULE(_hostbatch, m) {
  m.doc() = "C++ marshalling of pvt_place_host_batch (see csrc/pvt_hostpy.cpp)";
  m.def("place_host_batch", &place_host_batch, py::arg("fn"), py::arg("ctx"), py::arg("rounds"),
        py::arg("items"));
}
