// pybind11 bindings for the gfx950 device runtime (_hip).
//
// Every launcher takes raw device addresses (torch tensors' data_ptr()) and a
// raw hipStream_t (torch.cuda.current_stream().cuda_stream), so the module does
// not link libtorch: it shares torch's HIP runtime, allocator-owned buffers and
// streams, and keeps compile times at seconds.
#include <dlfcn.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "common.hpp"
#include "engine.hpp"
#include "exchange_sorted.hpp"
#include "ipc_comm.hpp"
#include "mailbox.hpp"
#include "server.hpp"
#include "xcall.hpp"
#include "gob_bridge.hpp"

namespace py = pybind11;

// roctx ranges for rocprofv3 --marker-trace, resolved at run time
// so the module has no hard dependency on the profiler SDK; no-ops without it.
namespace {
struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  void (*mark)(const char*) = nullptr;
  Roctx() {
    for (const char* lib : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4"}) {
      void* h = dlopen(lib, RTLD_NOW | RTLD_LOCAL);
      if (!h) continue;
      push = (int (*)(const char*))dlsym(h, "roctxRangePushA");
      pop = (int (*)())dlsym(h, "roctxRangePop");
      mark = (void (*)(const char*))dlsym(h, "roctxMarkA");
      if (push && pop) return;
    }
    push = nullptr;
    pop = nullptr;
    mark = nullptr;
  }
};
Roctx& roctx() {
  static Roctx r;
  return r;
}
}  // namespace

namespace ptype {
void launch_table_upsert(uintptr_t, uint64_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, int64_t,
                         uintptr_t, uintptr_t);
void launch_table_delete(uintptr_t, uint64_t, uintptr_t, int64_t, uintptr_t, uintptr_t, uintptr_t);
void launch_table_upsert_packed(uintptr_t, uint64_t, uintptr_t, uintptr_t, uintptr_t, int64_t, uintptr_t, uintptr_t);
void launch_table_lookup(uintptr_t, uint64_t, uintptr_t, int64_t, uintptr_t, uintptr_t, uintptr_t);
void launch_table_sweep(uintptr_t, uint64_t, uintptr_t, uint64_t, uintptr_t, uintptr_t);
void launch_table_pack(uintptr_t, uint64_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t);
void launch_gen_requests(uintptr_t, uintptr_t, uintptr_t, int64_t, uint32_t, uint64_t, uintptr_t, uintptr_t, bool);
void launch_replica_route(uintptr_t, uintptr_t, int64_t, const std::vector<int>&, uint64_t, uint32_t, uint32_t,
                          uintptr_t);
int replica_sel_max();
int64_t route_grid(int64_t, int64_t*);
int64_t gob_max_bytes(int64_t, int, uint32_t);
int64_t gob_ws_words(int64_t);
void launch_gob_encode(const std::vector<uintptr_t>&, int64_t, uint32_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t);
void launch_gob_decode(uintptr_t, uintptr_t, int64_t, uint32_t, const std::vector<uintptr_t>&, uintptr_t, uintptr_t);
void set_route_tuning(int, int, int);
int64_t route_fused_grid(int64_t, int64_t*);
void launch_table_build_dir(uintptr_t, uint64_t, uintptr_t, uint64_t, uint32_t, uintptr_t, uintptr_t, uintptr_t);
void launch_complete(uintptr_t, int64_t, uintptr_t, int64_t, uintptr_t, uintptr_t, uintptr_t, bool, uintptr_t, uintptr_t);
int64_t wire_req_words(int64_t, int, bool);
void launch_prime_gather(uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, int64_t, uintptr_t, uintptr_t, uintptr_t,
                         uintptr_t);
int64_t wire_rep_words(int64_t);
void launch_packed_meta(uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, int, int64_t, uint32_t, uint32_t,
                        uintptr_t, uintptr_t);
void launch_dispatch_packed(uintptr_t, int, int64_t, const PackedLayout&, uintptr_t, uintptr_t, uint32_t, uint64_t,
                            uintptr_t, int64_t, const std::vector<uintptr_t>&, uint64_t, const std::vector<uintptr_t>&,
                            int, uintptr_t);
void launch_complete_packed(uintptr_t, int64_t, int, int, uintptr_t, int64_t, uintptr_t, uintptr_t, uintptr_t, bool,
                            uintptr_t, uintptr_t, uintptr_t, int64_t);
void launch_records_to_soa(uintptr_t, int64_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, bool, uintptr_t);
void launch_snapshot_copy(uintptr_t, uintptr_t, int64_t, uintptr_t);
}  // namespace ptype

using namespace ptype;

static int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

static uintptr_t pinned_alloc(size_t bytes) {
  void* p = nullptr;
  PT_HIP_CHECK(hipHostMalloc(&p, bytes, hipHostMallocDefault));
  return (uintptr_t)p;
}
static void pinned_free(uintptr_t p) { PT_HIP_CHECK(hipHostFree((void*)p)); }

static void memcpy_d2h_async(uintptr_t dst, uintptr_t src, size_t bytes, uintptr_t stream) {
  PT_HIP_CHECK(hipMemcpyAsync((void*)dst, (const void*)src, bytes, hipMemcpyDeviceToHost, as_stream(stream)));
}
static void memcpy_h2d_async(uintptr_t dst, uintptr_t src, size_t bytes, uintptr_t stream) {
  PT_HIP_CHECK(hipMemcpyAsync((void*)dst, (const void*)src, bytes, hipMemcpyHostToDevice, as_stream(stream)));
}
static void stream_sync(uintptr_t stream) { PT_HIP_CHECK(hipStreamSynchronize(as_stream(stream))); }

namespace ptype {
void check_packed_layout(const PackedLayout& L, int R, int64_t C);
}

// v3 layouts cross the binding as dicts {off: [5], w: [5], S, vb}
static py::dict layout_dict(const PackedLayout& L) {
  py::dict d;
  d["off"] = std::vector<int>(L.off, L.off + 5);
  d["w"] = std::vector<int>(L.w, L.w + 5);
  d["S"] = (int)L.S;
  d["vb"] = (int)L.vb;
  return d;
}
static PackedLayout layout_of(const py::dict& d) {
  PackedLayout L{};
  const auto off = d["off"].cast<std::vector<int>>(), w = d["w"].cast<std::vector<int>>();
  if (off.size() != 5 || w.size() != 5) throw std::invalid_argument("layout: off and w need 5 entries");
  for (int q = 0; q < 5; ++q) {
    if (off[q] < 0 || off[q] > 255 || w[q] < 0 || w[q] > 64) throw std::invalid_argument("layout: bad field");
    L.off[q] = (uint8_t)off[q];
    L.w[q] = (uint8_t)w[q];
  }
  L.S = (uint8_t)d["S"].cast<int>();
  L.vb = (uint8_t)d["vb"].cast<int>();
  return L;
}

PYBIND11_MODULE(_hip, m) {
  m.doc() = "ptype_amd gfx950 device runtime: mailboxes, GPU registry, route/dispatch kernels";
  m.attr("ARCH") = "gfx950";
  m.attr("MSG_RECORD_BYTES") = (int)sizeof(MsgRecord);
  m.attr("REPLY_RECORD_BYTES") = (int)sizeof(ReplyRecord);
  m.attr("TABLE_ENTRY_BYTES") = (int)sizeof(TableEntry);
  m.attr("MAX_RANKS") = 64;
  m.def("device_count", &device_count);

  m.def("table_upsert", &launch_table_upsert, py::arg("table"), py::arg("cap"), py::arg("keys"),
        py::arg("ranks"), py::arg("mboxes"), py::arg("exp_in"), py::arg("exp_tbl"), py::arg("n"),
        py::arg("stats"), py::arg("stream"));
  m.def("table_upsert_packed", &launch_table_upsert_packed, py::arg("table"), py::arg("cap"), py::arg("entries"),
        py::arg("exp_in"), py::arg("exp_tbl"), py::arg("n"), py::arg("stats"), py::arg("stream"));
  m.def("table_delete", &launch_table_delete, py::arg("table"), py::arg("cap"), py::arg("keys"), py::arg("n"),
        py::arg("stats"), py::arg("found"), py::arg("stream"));
  m.def("table_lookup", &launch_table_lookup, py::arg("table"), py::arg("cap"), py::arg("keys"), py::arg("n"),
        py::arg("out_rank"), py::arg("out_mbox"), py::arg("stream"));
  m.def("table_sweep", &launch_table_sweep, py::arg("table"), py::arg("cap"), py::arg("exp_tbl"),
        py::arg("now"), py::arg("stats"), py::arg("stream"));
  m.def("table_pack", &launch_table_pack, py::arg("table"), py::arg("cap"), py::arg("exp_tbl"), py::arg("out"),
        py::arg("out_exp"), py::arg("out_count"), py::arg("stream"));

  // K4: gob value messages of fixed-schema int structs (csrc/hip/gob.hip)
  m.def("gob_max_bytes", &gob_max_bytes, py::arg("M"), py::arg("nf"), py::arg("type_id"));
  m.def("gob_ws_words", &gob_ws_words, py::arg("M"));
  m.def("gob_encode", &launch_gob_encode, py::arg("cols"), py::arg("M"), py::arg("type_id"), py::arg("out"),
        py::arg("offsets"), py::arg("ws"), py::arg("stream"));
  m.def("gob_decode", &launch_gob_decode, py::arg("buf"), py::arg("offsets"), py::arg("M"), py::arg("type_id"),
        py::arg("cols"), py::arg("status"), py::arg("stream"));
  m.def("gen_requests", &launch_gen_requests, py::arg("actor"), py::arg("a0"), py::arg("a1"), py::arg("M"),
        py::arg("n_actors"), py::arg("seed"), py::arg("seed_ptr"), py::arg("stream"), py::arg("wide") = false);
  m.def("replica_route", &launch_replica_route, py::arg("actor_in"), py::arg("actor_out"), py::arg("M"),
        py::arg("ranks"), py::arg("seq0"), py::arg("world"), py::arg("n_logical"), py::arg("stream"));
  m.def("max_replica_sel", &replica_sel_max);
  m.def("route_grid", [](int64_t M) {
    int64_t P;
    int64_t G = route_grid(M, &P);
    return py::make_tuple(G, P);
  });
  m.def("route", &launch_route, py::arg("actor"), py::arg("a0"), py::arg("a1"), py::arg("a2"),
        py::arg("method_col"), py::arg("method_uniform"), py::arg("M"), py::arg("table"), py::arg("cap"),
        py::arg("dir"), py::arg("n_dir"), py::arg("R"), py::arg("C"), py::arg("nargs"), py::arg("mc"),
        py::arg("sendbuf"), py::arg("perm"), py::arg("route"), py::arg("hist"), py::arg("lb"), py::arg("stats"),
        py::arg("rank_self"), py::arg("direct"), py::arg("affine_w"), py::arg("stream"));
  m.def("route_fused_grid", [](int64_t M) {
    int64_t P;
    const int64_t G = route_fused_grid(M, &P);
    return py::make_tuple(G, P);
  });
  m.def("wire_req_words", &wire_req_words, py::arg("C"), py::arg("nargs"), py::arg("mc"));
  m.def("wire_rep_words", &wire_rep_words, py::arg("C"));
  m.def("prime_gather", &launch_prime_gather, py::arg("val"), py::arg("st"), py::arg("first"), py::arg("n"),
        py::arg("target"), py::arg("T"), py::arg("out"), py::arg("out_st"), py::arg("scanned"), py::arg("stream"),
        "optimus watchReplies on the device: per target, the first non-target reply of its ranges (early exit)");
  m.def("roctx_available", [] { return roctx().push != nullptr; });
  m.def("roctx_push", [](const std::string& s) { return roctx().push ? roctx().push(s.c_str()) : -1; });
  m.def("roctx_pop", [] { return roctx().pop ? roctx().pop() : -1; });
  m.def("roctx_mark", [](const std::string& s) {
    if (roctx().mark) roctx().mark(s.c_str());
  });
  m.def("dp_ipc_transport", [] { return (uintptr_t)ipc_transport_ops(); },
        "the DpTransportOps table (csrc/core/dp_link.hpp) of IpcComm, for _core.DataPlane.use_transport");
  m.def(
      "host_comm_adopt",
      [](uintptr_t ref) {
        if (!ref) throw std::invalid_argument("host_comm_adopt: null reference");
        auto* p = reinterpret_cast<std::shared_ptr<HostComm>*>(ref);
        std::shared_ptr<HostComm> out = *p;
        delete p;
        return out;
      },
      py::arg("ref"), "the engines' communicator from DataPlane.engine_comm_ref() (one reference, adopted)");
  m.def("set_tune", &set_tune, py::arg("spec"),
        "apply 'key=value,...' path switches (csrc/hip/tune.hpp) after PTYPE_TUNE; false on an unknown key");
  m.def("tune", [] {
    const Tune t = tune();
    py::dict d;
    d["mbox_fused"] = t.mbox_fused, d["mbox_rec8"] = t.mbox_rec8, d["mbox_sort"] = t.mbox_sort;
    d["mbox_drain_msg"] = t.mbox_drain_msg, d["sx_sort"] = t.sx_sort, d["sx_self_copy"] = t.sx_self_copy;
    d["sx_comm_cs"] = t.sx_comm_cs, d["stream_sync"] = t.stream_sync;
    d["local"] = t.local, d["persistent_stream"] = t.persistent_stream, d["poll_lanes"] = t.poll_lanes;
    d["poll_full"] = t.poll_full, d["poll_sleep"] = t.poll_sleep;
    return d;
  }, "the native path switches in force");
  m.def("set_route_tuning", &set_route_tuning, py::arg("prep_items") = 0, py::arg("mode") = 0,
        py::arg("prep_pipe") = 0,
        "3-pass route_prep items per thread (1, 2, 4, 8; 0 = default); mode 0 = 3-pass prep/scan/scatter "
        "(default), 1 = single-pass look-back route; prep_pipe: 0 = default (directory path: next tile's ids "
        "loaded before this tile's gathers), -1 = off -- knobs for experiments");
  m.def("table_build_dir", &launch_table_build_dir, py::arg("table"), py::arg("cap"), py::arg("dir"),
        py::arg("n_dir"), py::arg("affine_w"), py::arg("affine_stats"), py::arg("stream"), py::arg("dir_rank") = 0,
        "K5b/K5c: the dense route directory (4-B route word per id) and, with dir_rank, its rank byte table");
  m.def("dispatch", &launch_dispatch, py::arg("recv"), py::arg("R"), py::arg("C"), py::arg("nargs"), py::arg("mc"),
        py::arg("reply"), py::arg("state"), py::arg("n_state"), py::arg("delay_ticks"), py::arg("stats"),
        py::arg("expected_per_rank"), py::arg("outbox"), py::arg("outbox_cap"), py::arg("direct"), py::arg("self"),
        py::arg("stream"));
  m.def("local_send", &launch_local_send, py::arg("actor"), py::arg("a0"), py::arg("a1"), py::arg("a2"),
        py::arg("method_col"), py::arg("method_uniform"), py::arg("M"), py::arg("table"), py::arg("cap"),
        py::arg("dir"), py::arg("n_dir"), py::arg("affine_w"), py::arg("state"), py::arg("n_state"),
        py::arg("delay_ticks"), py::arg("outbox"), py::arg("outbox_cap"), py::arg("out_val"), py::arg("out_status"),
        py::arg("stats"), py::arg("checksum"), py::arg("stream"), py::arg("m_dev") = 0,
        "world-1 Send: registry resolution + handler dispatch in one pass into the caller's outputs "
        "(m_dev: a device u64 holding the batch's real length <= M, read by the kernel)");
  m.def("outbox_seal", &launch_outbox_seal, py::arg("actor"), py::arg("cap"), py::arg("count"), py::arg("stream"),
        "before a device-counted multi-rank epoch: actor[i] = no-actor for min(count[0], cap) <= i < cap");
  m.def("outbox_advance", &launch_outbox_advance, py::arg("count"), py::arg("cap"), py::arg("epoch_m"), py::arg("j"),
        py::arg("stream"),
        "after a device-counted epoch: epoch_m[j] = min(count[0], cap), count[0] = 0 (the consumed bank)");
  m.def("complete", &launch_complete, py::arg("rep"), py::arg("C"), py::arg("perm"), py::arg("M"),
        py::arg("out_val"), py::arg("out_status"), py::arg("checksum"), py::arg("direct"), py::arg("stream"),
        py::arg("failed") = 0);
  m.def("records_to_soa", &launch_records_to_soa, py::arg("rec"), py::arg("M"), py::arg("actor"), py::arg("method"),
        py::arg("a0"), py::arg("a1"), py::arg("a2"), py::arg("mfma"), py::arg("stream"),
        "32-B AoS request records -> SoA columns (dwordx4 copy, or MFMA byte transposition)");
  m.def("snapshot_copy", &launch_snapshot_copy, py::arg("dst"), py::arg("src"), py::arg("n16"),
        py::arg("stream"));

  // ---- wire format v3 (packed.hpp): standalone kernels for tests and tools; the
  // epoch engine drives them itself (meta all-reduce + layout) in a Send
  m.attr("PACKED_META_WORDS") = (int)kMetaWords;
  m.def("packed_meta", &launch_packed_meta, py::arg("actor"), py::arg("a0"), py::arg("a1"), py::arg("a2"),
        py::arg("method_col"), py::arg("method_uniform"), py::arg("M"), py::arg("n_dir"), py::arg("affine_w"),
        py::arg("meta"), py::arg("stream"));
  m.def(
      "packed_layout",
      [](const std::vector<uint64_t>& meta) {
        if (meta.size() != (size_t)kMetaWords) throw std::invalid_argument("packed_layout: 16 meta words");
        return layout_dict(packed_layout(meta.data()));
      },
      py::arg("meta"));
  m.def("packed_reply_bits", [](const std::vector<uint64_t>& meta) {
    if (meta.size() != (size_t)kMetaWords) throw std::invalid_argument("packed_reply_bits: 16 meta words");
    return packed_reply_bits(meta.data());
  });
  m.def("packed_req_words", &packed_req_words, py::arg("C"), py::arg("S"));
  m.def("packed_rep_words", &packed_rep_words, py::arg("C"), py::arg("vb"));
  m.def(
      "route_packed",
      [](uintptr_t actor, uintptr_t a0, uintptr_t a1, uintptr_t a2, uintptr_t method_col, int method_uniform,
         int64_t M, uintptr_t table, uint64_t cap, uintptr_t dir, uint32_t n_dir, int R, int64_t C,
         const py::dict& layout, uintptr_t sendbuf, uintptr_t perm, uintptr_t route, uintptr_t hist, uintptr_t stats,
         int rank_self, const std::vector<uintptr_t>& direct, uint32_t affine_w, uintptr_t stream) {
        launch_route_packed(actor, a0, a1, a2, method_col, method_uniform, M, table, cap, dir, n_dir, R, C,
                            layout_of(layout), sendbuf, perm, route, hist, stats, rank_self, direct, affine_w, stream);
      },
      py::arg("actor"), py::arg("a0"), py::arg("a1"), py::arg("a2"), py::arg("method_col"), py::arg("method_uniform"),
      py::arg("M"), py::arg("table"), py::arg("cap"), py::arg("dir"), py::arg("n_dir"), py::arg("R"), py::arg("C"),
      py::arg("layout"), py::arg("sendbuf"), py::arg("perm"), py::arg("route"), py::arg("hist"), py::arg("stats"),
      py::arg("rank_self"), py::arg("direct"), py::arg("affine_w"), py::arg("stream"));
  m.def(
      "dispatch_packed",
      [](uintptr_t recv, int R, int64_t C, const py::dict& layout, uintptr_t reply, uintptr_t state, uint32_t n_state,
         uint64_t delay_ticks, uintptr_t stats, int64_t expected_per_rank, const std::vector<uintptr_t>& outbox,
         uint64_t outbox_cap, const std::vector<uintptr_t>& direct, int self, uintptr_t stream) {
        launch_dispatch_packed(recv, R, C, layout_of(layout), reply, state, n_state, delay_ticks, stats,
                               expected_per_rank, outbox, outbox_cap, direct, self, stream);
      },
      py::arg("recv"), py::arg("R"), py::arg("C"), py::arg("layout"), py::arg("reply"), py::arg("state"),
      py::arg("n_state"), py::arg("delay_ticks"), py::arg("stats"), py::arg("expected_per_rank"), py::arg("outbox"),
      py::arg("outbox_cap"), py::arg("direct"), py::arg("self"), py::arg("stream"));
  m.def("presence_words", &presence_words, py::arg("n_dir"),
        "int32 words of route mode 4's presence map for a directory of n_dir ids (0: too large for LDS)");
  m.def("presence_build", &launch_presence, py::arg("dir_rank"), py::arg("n_dir"), py::arg("rank"), py::arg("out"),
        py::arg("stream"), "route mode 4's presence map (2 bits per id: here / probe the table / not here) for rank");
  m.def("complete_packed", &launch_complete_packed, py::arg("rep"), py::arg("C"), py::arg("R"), py::arg("vb"), py::arg("perm"),
        py::arg("M"), py::arg("out_val"), py::arg("out_status"), py::arg("checksum"), py::arg("direct"),
        py::arg("stream"), py::arg("failed") = 0, py::arg("zero") = 0, py::arg("zero_words") = 0);

  m.def("pinned_alloc", &pinned_alloc);
  m.def("pinned_free", &pinned_free);
  m.def("memcpy_d2h_async", &memcpy_d2h_async);
  m.def("memcpy_h2d_async", &memcpy_h2d_async);
  m.def("stream_sync", &stream_sync, py::call_guard<py::gil_scoped_release>());

  py::class_<HostComm, std::shared_ptr<HostComm>>(m, "HostComm",
                                                  "a non-RCCL communicator the engines drive (FakeComm, IpcComm)")
      .def_property_readonly("size", &HostComm::size)
      .def_property_readonly("loopback", &HostComm::loopback)
      .def_property_readonly("device_side", &HostComm::device_side)
      .def("check", &HostComm::check, "raise if an earlier collective failed (a peer missed it)");
  py::class_<FakeComm, HostComm, std::shared_ptr<FakeComm>>(m, "FakeComm",
                                                            "in-process R-rank all-to-all for multi-rank engine tests "
                                                            "(one host thread + stream per rank on one GPU)")
      .def(py::init<int, bool, double>(), py::arg("R"), py::arg("loopback") = false, py::arg("link_gbps") = 0.0)
      .def(
          "allreduce_max",
          [](FakeComm& c, int rank, uintptr_t dev, int n, uintptr_t stream) {
            c.allreduce_max(rank, reinterpret_cast<uint64_t*>(dev), n, reinterpret_cast<hipStream_t>(stream));
          },
          py::arg("rank"), py::arg("dev"), py::arg("n"), py::arg("stream"), py::call_guard<py::gil_scoped_release>(),
          "element-wise max of n u64 over the in-process ranks (collective over them)");

  py::class_<IpcComm, HostComm, std::shared_ptr<IpcComm>>(
      m, "IpcComm",
      "one rank per PROCESS: collectives through shared-memory segments every rank maps and registers, "
      "stream-ordered on the device (csrc/hip/ipc_comm.hpp)")
      .def(py::init<int, int, int, size_t, double, const std::string&>(), py::arg("device"), py::arg("R"),
           py::arg("rank"), py::arg("cap_bytes"), py::arg("timeout_s"), py::arg("name"))
      .def("handle", &IpcComm::handle, "this rank's segment name")
      .def("connect", &IpcComm::connect, py::arg("names"))
      .def("seal", &IpcComm::seal, "remove this rank's segment name (after every rank connected)")
      .def_property_readonly("failed", &IpcComm::failed)
      .def_property_readonly("ops", &IpcComm::ops)
      .def_property_readonly("rank", &IpcComm::rank)
      .def_property_readonly("cap", &IpcComm::cap)
      .def(
          "alltoall",
          [](IpcComm& c, uintptr_t src, uintptr_t dst, size_t bytes, uintptr_t stream) {
            c.alltoall(c.rank(), (const void*)src, (void*)dst, bytes, reinterpret_cast<hipStream_t>(stream));
          },
          py::arg("src"), py::arg("dst"), py::arg("bytes"), py::arg("stream"))
      .def(
          "allreduce_max",
          [](IpcComm& c, uintptr_t dev, int n, uintptr_t stream) {
            c.allreduce_max(c.rank(), reinterpret_cast<uint64_t*>(dev), n, reinterpret_cast<hipStream_t>(stream));
          },
          py::arg("dev"), py::arg("n"), py::arg("stream"));

  py::class_<EpochEngine>(m, "EpochEngine",
                          "chunk-pipelined Send (route -> ncclAllToAll -> dispatch -> ncclAllToAll -> complete) "
                          "enqueued from one host call; comm = raw ncclComm_t or 0 for no collectives")
      .def(py::init<int, uintptr_t, int, int, int64_t, int64_t, int, std::shared_ptr<HostComm>, bool, int64_t>(),
           py::arg("device"), py::arg("comm"), py::arg("R"), py::arg("rank"), py::arg("C"), py::arg("max_chunk"),
           py::arg("chunks"), py::arg("fake") = nullptr, py::arg("adaptive") = false, py::arg("c_fixed") = 0)
      .def(
          "set_bufs",
          [](EpochEngine& e, int i, uintptr_t send, uintptr_t recv, uintptr_t reply, uintptr_t back, uintptr_t perm,
             uintptr_t src, uintptr_t route, uintptr_t hist, uintptr_t lb, uintptr_t ws) {
            e.set_bufs(i, EngineBufs{send, recv, reply, back, perm, src, route, hist, lb, ws});
          },
          py::arg("i"), py::arg("send"), py::arg("recv"), py::arg("reply"), py::arg("back"), py::arg("perm"),
          py::arg("src"), py::arg("route"), py::arg("hist"), py::arg("lb"), py::arg("ws"))
      .def(
          "send",
          [](EpochEngine& e, uintptr_t actor, uintptr_t a0, uintptr_t a1, uintptr_t a2, uintptr_t method_col,
             int method_uniform, int64_t M, uintptr_t table, uint64_t cap, uintptr_t dir, uint32_t n_dir,
             uint32_t affine_w, int nargs, bool mc, uintptr_t out_val, uintptr_t out_st, uintptr_t state,
             uint32_t n_state, uint64_t delay_ticks, const std::vector<uintptr_t>& outbox, uint64_t outbox_cap,
             bool direct, uintptr_t checksum, uintptr_t stream, bool packed, uintptr_t mailboxes, bool ordered,
             uintptr_t m_dev) {
            e.send(EngineSend{actor, a0, a1, a2, method_col, method_uniform, M, table, cap, dir, n_dir, affine_w,
                              nargs, mc, out_val, out_st, state, n_state, delay_ticks, outbox, outbox_cap, direct,
                              checksum, stream, packed, mailboxes, ordered, m_dev});
          },
          py::arg("actor"), py::arg("a0"), py::arg("a1"), py::arg("a2"), py::arg("method_col"),
          py::arg("method_uniform"), py::arg("M"), py::arg("table"), py::arg("cap"), py::arg("dir"), py::arg("n_dir"),
          py::arg("affine_w"), py::arg("nargs"), py::arg("mc"), py::arg("out_val"), py::arg("out_st"),
          py::arg("state"), py::arg("n_state"), py::arg("delay_ticks"), py::arg("outbox"), py::arg("outbox_cap"),
          py::arg("direct"), py::arg("checksum"), py::arg("stream"), py::arg("packed") = false,
          py::arg("mailboxes") = 0, py::arg("ordered") = false, py::arg("m_dev") = 0,
          py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("stream_values", &EpochEngine::stream_values)
      .def("hang_state", &EpochEngine::hang_state, py::arg("compute_stream"))
      .def("last_wire",
           [](const EpochEngine& e) {
             const auto& w = e.last_wire();
             py::dict d = layout_dict(w.layout);
             d["req_words"] = w.req_words;
             d["rep_words"] = w.rep_words;
             d["C"] = w.C;
             d["C_alloc"] = w.C_alloc;
             d["adapted"] = w.adapted;
             d["exact"] = w.exact;
             d["meta"] = std::vector<uint64_t>(w.meta, w.meta + kMetaWords);
             return d;
           },
           "wire format of the last send: v3 layout (S == 0: v2), words per chunk on each all-to-all")
      .def("host_profile",
           [](const EpochEngine& e) {
             const auto p = e.host_profile();
             py::dict d;
             d["sends"] = p.sends;
             d["kernels_ns"] = p.kernels_ns;
             d["a2a_ns"] = p.a2a_ns;
             d["sync_ns"] = p.sync_ns;
             d["meta_ns"] = p.meta_ns;
             d["total_ns"] = p.total_ns;
             return d;
           })
      .def("reset_host_profile", &EpochEngine::reset_host_profile);
  py::class_<SortedExchange>(m, "SortedExchange",
                             "multi-GPU Send with mailbox delivery: the sender's counting sort by (rank, actor shard) "
                             "fills the peers' mailboxes directly; see csrc/hip/exchange_sorted.hpp")
      .def(py::init<int, uintptr_t, int, int, int64_t, int, int64_t, int64_t, std::shared_ptr<HostComm>>(),
           py::arg("device"), py::arg("comm"), py::arg("R"), py::arg("rank"), py::arg("max_chunk"), py::arg("chunks"),
           py::arg("C_alloc"), py::arg("C0"), py::arg("fake") = nullptr)
      .def(
          "send",
          [](SortedExchange& e, uintptr_t actor, uintptr_t a0, uintptr_t a1, uintptr_t a2, uintptr_t method_col,
             int method_uniform, int64_t M, uintptr_t table, uint64_t cap, uintptr_t dir, uint32_t n_dir,
             uint32_t affine_w, uintptr_t out_val, uintptr_t out_st, uintptr_t state, uint32_t n_state,
             uint64_t delay_ticks, bool ordered, uintptr_t stream, uintptr_t dir_rank) {
            SxSend a;
            a.actor = actor, a.a0 = a0, a.a1 = a1, a.a2 = a2, a.method_col = method_col;
            a.method_uniform = method_uniform, a.M = M, a.table = table, a.cap = cap, a.dir = dir, a.n_dir = n_dir;
            a.affine_w = affine_w, a.out_val = out_val, a.out_st = out_st, a.state = state, a.n_state = n_state;
            a.delay_ticks = delay_ticks, a.ordered = ordered, a.stream = stream, a.dir_rank = dir_rank;
            e.send(a);
          },
          py::arg("actor"), py::arg("a0"), py::arg("a1"), py::arg("a2"), py::arg("method_col"),
          py::arg("method_uniform"), py::arg("M"), py::arg("table"), py::arg("cap"), py::arg("dir"), py::arg("n_dir"),
          py::arg("affine_w"), py::arg("out_val"), py::arg("out_st"), py::arg("state"), py::arg("n_state"),
          py::arg("delay_ticks"), py::arg("ordered"), py::arg("stream"), py::arg("dir_rank") = 0,
          py::call_guard<py::gil_scoped_release>())
      .def("last_wire",
           [](const SortedExchange& e) {
             const auto& w = e.last_wire();
             py::dict d = layout_dict(w.L);
             d["S"] = w.S;  // as moved (the layout's dwords rounded to a kernel variant)
             d["req_words"] = w.req_words;
             d["rep_words"] = w.rep_words;
             d["req_moved"] = w.req_moved;
             d["rep_moved"] = w.rep_moved;
             d["pairs"] = w.pairs;
             d["cap_out"] = std::vector<uint32_t>(w.cap_out, w.cap_out + e.ranks());
             d["cap_in"] = std::vector<uint32_t>(w.cap_in, w.cap_in + e.ranks());
             d["C"] = w.C;
             d["agreed"] = w.agreed;
             d["spec_from"] = w.spec_from;
             d["shard_ok"] = w.shard_ok;
             d["route_mode"] = w.route_mode;
             d["meta"] = std::vector<uint64_t>(w.meta, w.meta + kMetaWords);
             return d;
           },
           "geometry of the last send (region strides per peer and chunk; *_moved: words this rank sent per "
           "chunk, all peers; pairs: per-pair capacities in force); agreed: from the agreement of Send spec_from")
      .def("stats", &SortedExchange::stats)
      .def_property("epoch_counter", &SortedExchange::epoch_counter, &SortedExchange::set_epoch_counter)
      .def("last_overflow", &SortedExchange::last_overflow, py::call_guard<py::gil_scoped_release>(),
           "messages the last Send answered STATUS_OVERFLOW, max over ranks (waits for its agreement copy)")
      .def("overflow_of", &SortedExchange::overflow_of, py::arg("send"), py::call_guard<py::gil_scoped_release>(),
           "the same count for Send `send` (valid until Send send + 2 is issued)")
      .def("host_profile",
           [](const SortedExchange& e) {
             const auto p = e.host_profile();
             py::dict d;
             d["sends"] = p.sends;
             d["total_ns"] = p.total_ns;
             d["spec_wait_ns"] = p.spec_wait_ns;
             d["overflow_waits"] = p.overflow_waits;
             d["overflow_wait_ns"] = p.overflow_wait_ns;
             return d;
           },
           "host time of send() calls; spec_wait_ns: waits for Send k - 2's agreement (backpressure); "
           "overflow_waits: reads of a Send's overflow count (last_overflow / overflow_of)")
      .def_property_readonly("sends", &SortedExchange::sends);
  py::class_<Mailboxes>(m, "Mailboxes",
                        "HBM actor mailboxes: S shard rings of Q 32-B tagged records (K2 enqueue, K3 epoch drain, "
                        "K3 persistent consumer); see csrc/hip/mailbox.hpp")
      .def(py::init<int, uint32_t, uint32_t, bool>(), py::arg("device"), py::arg("shards") = 256,
           py::arg("slots") = 65536, py::arg("with_a2") = true)
      .def("enqueue", &Mailboxes::enqueue, py::arg("actor"), py::arg("a0"), py::arg("a1"), py::arg("a2"),
           py::arg("method_col"), py::arg("method_uniform"), py::arg("M"), py::arg("table"), py::arg("cap"),
           py::arg("dir"), py::arg("n_dir"), py::arg("affine_w"), py::arg("rank_self"), py::arg("origin_base"),
           py::arg("out_val"), py::arg("out_st"), py::arg("out_n"), py::arg("live"), py::arg("stream"),
           py::arg("arrival") = false)
      .def("drain", &Mailboxes::drain, py::arg("state"), py::arg("n_state"), py::arg("delay_ticks"),
           py::arg("out_val"), py::arg("out_st"), py::arg("out_n"), py::arg("ordered"), py::arg("stream"),
           py::arg("outbox") = std::vector<uintptr_t>{}, py::arg("outbox_cap") = 0, py::arg("fixed_method") = 0)
      .def(
          "send_sorted",
          [](Mailboxes& mb, uintptr_t actor, uintptr_t a0, uintptr_t a1, uintptr_t a2, uintptr_t method_col,
             int method_uniform, int64_t M, uintptr_t table, uint64_t cap, uintptr_t dir, uint32_t n_dir,
             uint32_t affine_w, int rank_self, uint32_t origin_base, uintptr_t out_val, uintptr_t out_st,
             uint64_t out_n, uintptr_t state, uint32_t n_state, uint64_t delay_ticks,
             const std::vector<uintptr_t>& outbox, uint64_t outbox_cap, bool arrival, bool ordered,
             int fixed_method, uintptr_t stream, int sort_mode, uintptr_t dir_rank, uintptr_t pres, int pres_rank) {
            MboxSend a;
            a.actor = actor, a.a0 = a0, a.a1 = a1, a.a2 = a2, a.method_col = method_col;
            a.method_uniform = method_uniform, a.M = M, a.table = table, a.cap = cap, a.dir = dir;
            a.n_dir = n_dir, a.affine_w = affine_w, a.rank_self = rank_self, a.origin_base = origin_base;
            a.out_val = out_val, a.out_st = out_st, a.out_n = out_n, a.state = state, a.n_state = n_state;
            a.delay_ticks = delay_ticks, a.outbox = outbox, a.outbox_cap = outbox_cap, a.arrival = arrival;
            a.ordered = ordered, a.fixed_method = fixed_method, a.stream = stream, a.sort_mode = sort_mode;
            a.dir_rank = dir_rank, a.pres = pres, a.pres_rank = pres_rank;
            mb.send_sorted(a);
          },
          "epoch Send through the sorted mailboxes: stable counting-sort enqueue + ordered / parallel drain",
          py::arg("actor"), py::arg("a0"), py::arg("a1"), py::arg("a2"), py::arg("method_col"),
          py::arg("method_uniform"), py::arg("M"), py::arg("table"), py::arg("cap"), py::arg("dir"), py::arg("n_dir"),
          py::arg("affine_w"), py::arg("rank_self"), py::arg("origin_base"), py::arg("out_val"), py::arg("out_st"),
          py::arg("out_n"), py::arg("state"), py::arg("n_state"), py::arg("delay_ticks"), py::arg("outbox"),
          py::arg("outbox_cap"), py::arg("arrival"), py::arg("ordered"), py::arg("fixed_method"), py::arg("stream"),
          py::arg("sort_mode") = 0, py::arg("dir_rank") = 0, py::arg("pres") = 0, py::arg("pres_rank") = -1)
      .def("start", &Mailboxes::start, py::arg("state"), py::arg("n_state"), py::arg("delay_ticks"),
           py::arg("out_val"), py::arg("out_st"), py::arg("out_n"), py::arg("blocks") = 16, py::arg("idle_ms") = 0.0,
           py::arg("max_s") = 60.0)
      .def("stop", &Mailboxes::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("running", &Mailboxes::running)
      .def("reset", &Mailboxes::reset, py::arg("stream"))
      .def("stats", &Mailboxes::stats)
      .def_property("epoch_counter", &Mailboxes::epoch_counter, &Mailboxes::set_epoch_counter)
      .def("shard_counters", &Mailboxes::shard_counters)
      .def_property_readonly("shards", &Mailboxes::shards)
      .def_property_readonly("slots", &Mailboxes::slots)
      .def_property_readonly("bytes", &Mailboxes::bytes)
      .def_property_readonly("last_record_bytes", &Mailboxes::last_record_bytes)
      .def_property_readonly("last_view_shards", &Mailboxes::last_view_shards)
      .def_property_readonly("last_route", &Mailboxes::last_route)
      .def_property_readonly("consumer_processed", &Mailboxes::consumer_processed)
      .def_property_readonly("launches", &Mailboxes::launches)
      .def_property_readonly("handle", [](Mailboxes& m) { return (uintptr_t)&m; },
                             "address of the C++ object (the epoch engine delivers into these mailboxes)");
  m.def("rccl_available", [] { return rccl().alltoall != nullptr; });

  py::class_<GobBridge>(m, "GobBridge",
                        "K4 on the net/rpc serving path: batched gob requests decoded on the GPU into mailbox "
                        "columns (csrc/hip/gob_bridge.hpp); pass handle() to RpcServer.register_device_batch")
      .def(py::init([](int device, Mailboxes& mb, uint32_t method, uint32_t fixed_actor, uintptr_t table,
                       uint64_t cap, uintptr_t state, uint32_t n_state, uint64_t delay_us, uintptr_t order_stream) {
             return new GobBridge(device, &mb, method, fixed_actor, table, cap, state, n_state, delay_us * 100,
                                  order_stream);
           }),
           py::arg("device"), py::arg("mailboxes"), py::arg("method"), py::arg("actor") = 0, py::arg("table"),
           py::arg("cap"), py::arg("state") = 0, py::arg("n_state") = 0, py::arg("delay_us") = 0,
           py::arg("order_stream") = 0, py::keep_alive<1, 3>())
      .def("retarget", &GobBridge::retarget, py::arg("table"), py::arg("cap"), py::arg("state"), py::arg("n_state"),
           py::call_guard<py::gil_scoped_release>())
      .def("handle", [](GobBridge& b) {
        return py::make_tuple((uintptr_t)&GobBridge::batch_c, (uintptr_t)&b);
      })
      .def_property_readonly("batches", &GobBridge::batches)
      .def_property_readonly("calls", &GobBridge::calls);
  py::class_<PeerLane, std::shared_ptr<PeerLane>>(m, "PeerLane")
      .def(py::init([](const std::string& shm, int device, double timeout_s) {
             py::gil_scoped_release nogil;
             return std::make_shared<PeerLane>(shm, device, timeout_s);
           }),
           py::arg("shm_name"), py::arg("device"), py::arg("timeout_s") = 10.0)
      .def("call", &PeerLane::call, py::arg("actor"), py::arg("method"), py::arg("method_uniform"), py::arg("a0"),
           py::arg("a1"), py::arg("a2"), py::arg("n"), py::arg("out_val"), py::arg("out_st"), py::arg("ticks"),
           py::arg("timeout_s"), py::arg("stream"), py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("lane", &PeerLane::lane)
      .def_property_readonly("calls", &PeerLane::calls);
  py::class_<PeerRelay, std::shared_ptr<PeerRelay>>(m, "PeerRelay",
                                                    "handler-initiated remote calls: peer lanes on another "
                                                    "dispatcher as a relay table for this process's dispatcher")
      .def(py::init([](const std::string& shm, int device, int n_lanes, double timeout_s) {
             py::gil_scoped_release nogil;
             return std::make_shared<PeerRelay>(shm, device, n_lanes, timeout_s);
           }),
           py::arg("shm_name"), py::arg("device"), py::arg("n_lanes") = 8, py::arg("timeout_s") = 1.0)
      .def_property_readonly("table", &PeerRelay::table)
      .def_property_readonly("lanes", &PeerRelay::lanes)
      .def("slots", &PeerRelay::slots, "per lane [seq, suspect] as the device table holds them");
  py::class_<DeviceServer>(m, "DeviceServer")
      .def(py::init<int, uint32_t, uintptr_t, uint32_t, uint64_t, double, double, const std::string&>(),
           py::arg("device"), py::arg("ring") = 4096, py::arg("state") = 0, py::arg("n_state") = 0,
           py::arg("delay_us") = 0, py::arg("idle_ms") = 200.0, py::arg("max_s") = 60.0, py::arg("shm_name") = "")
      .def("export_method", &DeviceServer::export_method, py::arg("name"), py::arg("method"), py::arg("actor") = 0,
           py::arg("fields") = std::vector<std::string>{}, py::arg("actor_field") = "")
      .def_property_readonly("shm_name", &DeviceServer::shm_name)
      .def_property_readonly("xlanes", [](DeviceServer& s) { return s.xlanes_exported(); })
      .def("set_relay", &DeviceServer::set_relay, py::arg("table"),
           "route kMethodRelay calls through a PeerRelay's table (0: off)")
      .def(
          "call",
          [](DeviceServer& s, int method, uint32_t actor, int64_t a0, int64_t a1, int64_t a2, double timeout) {
            MsgRecord m{actor, (uint16_t)method, (uint16_t)kFlagValid, a0, a1, a2};
            ReplyRecord r;
            {
              py::gil_scoped_release nogil;
              s.call(&m, &r, 1, timeout);
            }
            return py::make_tuple(r.value, r.status, r.actor);
          },
          py::arg("method"), py::arg("actor"), py::arg("a0") = 0, py::arg("a1") = 0, py::arg("a2") = 0,
          py::arg("timeout") = 30.0)
      .def(
          "call_many",
          [](DeviceServer& s, uintptr_t req, uintptr_t rep, int n, double timeout) {
            py::gil_scoped_release nogil;
            s.call((const MsgRecord*)req, (ReplyRecord*)rep, n, timeout);
          },
          py::arg("req"), py::arg("rep"), py::arg("n"), py::arg("timeout") = 30.0)
      .def("close", &DeviceServer::close, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("processed", &DeviceServer::processed)
      .def_property_readonly("ring_on_device", &DeviceServer::ring_on_device)
      .def_property_readonly("ring_fds_handed", &DeviceServer::ring_fds_handed)
      .def_property_readonly("stream_priority", &DeviceServer::stream_priority)
      .def_property_readonly("launches", &DeviceServer::launches)
      .def_property_readonly("exits_idle", &DeviceServer::exits_idle)
      .def_property_readonly("exits_lifetime", &DeviceServer::exits_lifetime)
      .def_property_readonly("running", &DeviceServer::running)
      .def("enable_trace", &DeviceServer::enable_trace, py::arg("capacity") = 4096)
      .def("disable_trace", &DeviceServer::disable_trace)
      .def("trace_records",
           [](const DeviceServer& s) {
             const auto v = s.trace_records();
             return py::bytes(reinterpret_cast<const char*>(v.data()), v.size() * sizeof(TraceRec));
           },
           "raw TraceRec ring: uint64 [seq, t_pub_ns, t_seen_ticks, t_done_ticks] per record")
      .def("calibrate", &DeviceServer::calibrate, py::arg("timeout") = 2.0,
           py::call_guard<py::gil_scoped_release>(), "[host_ns, device_ticks, half_window_ns]")
      .def("rtt_histogram", &DeviceServer::rtt_histogram, "host round-trip counts per log2(ns) bucket")
      .def_static("now_ns", &DeviceServer::now_ns)
      .def("submit_handle", [](DeviceServer& s) {
        return py::make_tuple((uintptr_t)&DeviceServer::submit_c, (uintptr_t)&s);
      });
}
