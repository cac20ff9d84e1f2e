// pybind11 module `_runtime`: the host-native runtime of the swarm node.
//
// Pure C++ (no torch, no HIP): cache layout + swarm directory + exchange planner, the
// origin packager (TS mux + AES-128-CBC), and CPU reference implementations of every
// device kernel (decrypt, demux, CRC) used as test oracles and by the CPU (no-GPU) mode.
// Batch entry points take numpy arrays (torch CPU tensors pass via .numpy()).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <sstream>
#include <stdexcept>
#include <thread>
#include <tuple>
#include <vector>

#include "aes_host.hpp"
#include "crc_host.hpp"
#include "locator.hpp"
#include "planner.hpp"
#include "shm_control.hpp"
#include "store.hpp"
#include "ts.hpp"
#include "wants.hpp"

namespace py = pybind11;
using namespace hlsp2p;

namespace {

template <typename T>
using Arr = py::array_t<T, py::array::c_style | py::array::forcecast>;

template <typename T>
T* mut_ptr(py::array& a, const char* name) {
  if (!(a.flags() & py::array::c_style)) throw std::invalid_argument(std::string(name) + " must be C-contiguous");
  if (a.itemsize() != sizeof(T)) throw std::invalid_argument(std::string(name) + " has the wrong dtype");
  if (!a.writeable()) throw std::invalid_argument(std::string(name) + " must be writeable");
  return static_cast<T*>(a.mutable_data());
}

template <typename F>
void parallel_for(int64_t n, F&& f, int64_t work_bytes = -1) {
  unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  int64_t nt = std::min<int64_t>(n, std::min<unsigned>(hw, 16u));
  // a thread spawn costs ~10-20 us: small batches (host-path probes, unit tests) run inline
  if (work_bytes >= 0) nt = std::min<int64_t>(nt, std::max<int64_t>(1, work_bytes >> 20));
  if (nt <= 1) {
    for (int64_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::vector<std::thread> th;
  for (int64_t t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      for (int64_t i = t; i < n; i += nt) f(i);
    });
  for (auto& x : th) x.join();
}

SegKey key_from(const int64_t* p) {
  return SegKey{uint32_t(p[0]), uint32_t(p[1]), uint32_t(p[2]), uint32_t(p[3])};
}

py::array_t<uint8_t> to_u8(const std::vector<uint8_t>& v) {
  py::array_t<uint8_t> a(static_cast<py::ssize_t>(v.size()));
  std::memcpy(a.mutable_data(), v.data(), v.size());
  return a;
}

}  // namespace

namespace {
// Replicated swarm state that differs across ranks (directory content or a round's plan).
struct SwarmDivergence : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// "digest A: ranks [0, 1, 2]; digest B: ranks [3]" for one header word of every rank
std::string group_ranks(const std::vector<Arr<int64_t>>& parts, int64_t word) {
  std::map<int64_t, std::vector<int>> by;
  for (size_t r = 0; r < parts.size(); ++r) by[parts[r].data()[word]].push_back(int(r));
  std::ostringstream o;
  bool first = true;
  for (const auto& kv : by) {
    o << (first ? "" : "; ") << std::hex << "0x" << uint64_t(kv.first) << std::dec << ": ranks [";
    for (size_t i = 0; i < kv.second.size(); ++i) o << (i ? ", " : "") << kv.second[i];
    o << "]";
    first = false;
  }
  return o.str();
}
}  // namespace

PYBIND11_MODULE(_runtime, m) {
  py::register_exception<SwarmDivergence>(m, "SwarmDivergence", PyExc_RuntimeError);
  m.doc() = "hlsjs-p2p-wrapper-amd host runtime (store, planner, packager, CPU oracles)";

  // ------------------------------------------------------------------ AES
  m.def("aes_tables", [] {
    const aes::Tables& t = aes::tables();
    Arr<uint32_t> td0(256), te0(256);
    Arr<uint8_t> sbox(256), inv(256);
    std::memcpy(td0.mutable_data(), t.td0, sizeof t.td0);
    std::memcpy(te0.mutable_data(), t.te0, sizeof t.te0);
    std::memcpy(sbox.mutable_data(), t.sbox, 256);
    std::memcpy(inv.mutable_data(), t.inv_sbox, 256);
    return py::make_tuple(td0, inv, te0, sbox);
  });
  m.def("expand_key_dec", [](py::bytes key) {
    std::string k = key;
    if (k.size() != 16) throw std::invalid_argument("AES-128 key must be 16 bytes");
    Arr<uint32_t> out(44);
    aes::expand_key_dec(reinterpret_cast<const uint8_t*>(k.data()), out.mutable_data());
    return out;
  });
  m.def("expand_key_enc", [](py::bytes key) {
    std::string k = key;
    if (k.size() != 16) throw std::invalid_argument("AES-128 key must be 16 bytes");
    Arr<uint32_t> out(44);
    aes::expand_key_enc(reinterpret_cast<const uint8_t*>(k.data()), out.mutable_data());
    return out;
  });
  m.def("aes_encrypt_block", [](py::bytes key, py::bytes block) {
    std::string k = key, b = block;
    if (k.size() != 16 || b.size() != 16) throw std::invalid_argument("16-byte key and block");
    uint32_t rk[44];
    aes::expand_key_enc(reinterpret_cast<const uint8_t*>(k.data()), rk);
    uint8_t out[16];
    aes::encrypt_block(rk, reinterpret_cast<const uint8_t*>(b.data()), out);
    return py::bytes(reinterpret_cast<char*>(out), 16);
  });
  m.def("cbc_encrypt", [](py::bytes key, py::bytes iv, Arr<uint8_t> data) {
    std::string k = key, v = iv;
    if (k.size() != 16 || v.size() != 16) throw std::invalid_argument("16-byte key and iv");
    const size_t n = static_cast<size_t>(data.size());
    std::vector<uint8_t> out(n + 16);
    size_t total;
    {
      py::gil_scoped_release nogil;
      total = aes::cbc_encrypt_pkcs7(reinterpret_cast<const uint8_t*>(k.data()),
                                     reinterpret_cast<const uint8_t*>(v.data()), data.data(), n, out.data());
    }
    out.resize(total);
    return to_u8(out);
  });
  m.def("cbc_decrypt", [](py::bytes key, py::bytes iv, Arr<uint8_t> data) -> py::object {
    std::string k = key, v = iv;
    if (k.size() != 16 || v.size() != 16) throw std::invalid_argument("16-byte key and iv");
    const size_t n = static_cast<size_t>(data.size());
    std::vector<uint8_t> out(n);
    int64_t len;
    {
      py::gil_scoped_release nogil;
      len = aes::cbc_decrypt_pkcs7(reinterpret_cast<const uint8_t*>(k.data()),
                                   reinterpret_cast<const uint8_t*>(v.data()), data.data(), n, out.data());
    }
    if (len < 0) return py::none();
    out.resize(static_cast<size_t>(len));
    return to_u8(out);
  });
  // Batched CPU decrypt with the device kernel's argument layout.
  //   src/dst: flat uint8; src_off/dst_off/nbytes: int64[B]; drk: uint32[B,44]; iv: uint8[B,16]
  //   out_len: int64[B] (plaintext length after PKCS#7, -1 on bad padding)
  m.def("cbc_decrypt_batch", [](Arr<uint8_t> src, py::array dst, Arr<int64_t> src_off, Arr<int64_t> dst_off,
                                Arr<int64_t> nbytes, Arr<uint32_t> drk, Arr<uint8_t> iv, py::array out_len) {
    const int64_t B = src_off.size();
    uint8_t* d = mut_ptr<uint8_t>(dst, "dst");
    int64_t* ol = mut_ptr<int64_t>(out_len, "out_len");
    const uint8_t* s = src.data();
    const int64_t* so = src_off.data();
    const int64_t* dof = dst_off.data();
    const int64_t* nb = nbytes.data();
    const uint32_t* k = drk.data();
    const uint8_t* ivp = iv.data();
    const int64_t src_n = src.size(), dst_n = dst.size();
    for (int64_t b = 0; b < B; ++b)
      if (nb[b] < 0 || nb[b] % 16 || so[b] < 0 || so[b] + nb[b] > src_n || dof[b] < 0 || dof[b] + nb[b] > dst_n)
        throw std::invalid_argument("cbc_decrypt_batch: segment out of bounds or not a multiple of 16");
    int64_t total = 0;
    for (int64_t b = 0; b < B; ++b) total += nb[b];
    py::gil_scoped_release nogil;
    parallel_for(B, [&](int64_t b) {
      uint8_t* out = d + dof[b];
      aes::cbc_decrypt_raw(k + 44 * b, ivp + 16 * b, s + so[b], static_cast<size_t>(nb[b]), out);
      int64_t len = -1;
      if (nb[b] >= 16) {
        uint8_t pad = out[nb[b] - 1];
        if (pad >= 1 && pad <= 16) {
          len = nb[b] - pad;
          for (int64_t i = len; i < nb[b]; ++i)
            if (out[i] != pad) { len = -1; break; }
        }
      }
      ol[b] = len;
    }, total);
  });

  // ------------------------------------------------------------------ CRC
  m.def("crc32", [](Arr<uint8_t> data, uint32_t crc) {
    return crc::crc32(data.data(), static_cast<size_t>(data.size()), crc);
  }, py::arg("data"), py::arg("crc") = 0u);
  m.def("crc32_batch", [](Arr<uint8_t> buf, Arr<int64_t> off, Arr<int64_t> len) {
    const int64_t B = off.size();
    Arr<uint32_t> out(B);
    uint32_t* o = out.mutable_data();
    const uint8_t* p = buf.data();
    const int64_t* of = off.data();
    const int64_t* ln = len.data();
    for (int64_t b = 0; b < B; ++b)
      if (of[b] < 0 || ln[b] < 0 || of[b] + ln[b] > buf.size()) throw std::invalid_argument("crc32_batch: out of bounds");
    int64_t total = 0;
    for (int64_t b = 0; b < B; ++b) total += ln[b];
    py::gil_scoped_release nogil;
    parallel_for(B, [&](int64_t b) { o[b] = crc::crc32(p + of[b], static_cast<size_t>(ln[b])); }, total);
    return out;
  });
  m.def("crc_mfma_weights", [] {
    auto w = crc::mfma_group_weights();
    Arr<int8_t> a(static_cast<py::ssize_t>(w.size()));
    std::memcpy(a.mutable_data(), w.data(), w.size());
    return a;
  });
  m.def("crc_mfma_weights_fp4", [] {
    auto w = crc::mfma_group_weights_fp4();
    Arr<uint8_t> a(static_cast<py::ssize_t>(w.size()));
    std::memcpy(a.mutable_data(), w.data(), w.size());
    return a;
  });
  m.def("crc_chunk_weights_fp4", [] {
    auto w = crc::mfma_chunk_weights_fp4();
    Arr<uint8_t> a(static_cast<py::ssize_t>(w.size()));
    std::memcpy(a.mutable_data(), w.data(), w.size());
    return a;
  });
  m.def("crc_init_fold", &crc::init_fold, py::arg("nbytes"));
  m.def("crc_shift_tables", [] {
    auto t = crc::shift_tables();
    Arr<uint32_t> a(static_cast<py::ssize_t>(t.size()));
    std::memcpy(a.mutable_data(), t.data(), t.size() * 4);
    return a;
  });
  m.attr("CRC_NUM_P") = crc::kNumP;
  m.attr("CRC_NUM_Q") = crc::kNumQ;
  m.attr("CRC_GROUP_BYTES") = crc::kGroupBytes;
  m.attr("CRC_CHUNK_BYTES") = crc::kChunkBytes;
  m.attr("CRC_FUSED_AES_STEPS") = crc::kFusedAesSteps;
  m.attr("CRC_FUSED_FOLD_STEPS") = crc::kFusedFoldSteps;
  m.attr("CRC_FUSED_MASK_DWORDS") = crc::kFusedMaskDwords;

  // ------------------------------------------------------------------ TS
  m.def("mux_segment", [](double duration, double fps, int64_t target_bytes, int audio_kbps, bool with_id3,
                          uint64_t seed, int64_t sn, double start_time) {
    ts::MuxConfig c;
    c.duration = duration; c.fps = fps; c.target_bytes = target_bytes; c.audio_kbps = audio_kbps;
    c.with_id3 = with_id3; c.seed = seed; c.sn = sn; c.start_time = start_time;
    ts::MuxStats st;
    std::vector<uint8_t> v;
    {
      py::gil_scoped_release nogil;
      v = ts::mux_segment(c, &st);
    }
    py::dict d;
    d["es_bytes"] = py::make_tuple(st.es_bytes[0], st.es_bytes[1], st.es_bytes[2]);
    d["n_pes"] = py::make_tuple(st.n_pes[0], st.n_pes[1], st.n_pes[2]);
    d["first_pts"] = py::make_tuple(st.first_pts[0], st.first_pts[1], st.first_pts[2]);
    d["last_pts"] = py::make_tuple(st.last_pts[0], st.last_pts[1], st.last_pts[2]);
    d["n_packets"] = st.n_packets;
    return py::make_tuple(to_u8(v), d);
  }, py::arg("duration"), py::arg("fps"), py::arg("target_bytes"), py::arg("audio_kbps"), py::arg("with_id3"),
     py::arg("seed"), py::arg("sn"), py::arg("start_time"));
  // Batched CPU demux with the device kernels' layout.
  //   buf: flat uint8 plaintext; off/len: int64[B]; es: flat uint8 (segment b writes at es_off[b])
  //   pes: int64[B, 3, max_pes, 3]; info: int64[B, 16]
  m.def("demux_batch", [](Arr<uint8_t> buf, Arr<int64_t> off, Arr<int64_t> len, py::array es, Arr<int64_t> es_off,
                          py::array pes, py::array info, int64_t max_pes) {
    const int64_t B = off.size();
    uint8_t* e = mut_ptr<uint8_t>(es, "es");
    int64_t* pp = mut_ptr<int64_t>(pes, "pes");
    int64_t* ip = mut_ptr<int64_t>(info, "info");
    if (pes.size() < B * ts::kClasses * max_pes * 3 || info.size() < B * ts::kInfoWords)
      throw std::invalid_argument("demux_batch: pes/info too small");
    for (int64_t b = 0; b < B; ++b)
      if (off.data()[b] < 0 || len.data()[b] < 0 || off.data()[b] + len.data()[b] > buf.size() ||
          es_off.data()[b] < 0 || es_off.data()[b] + len.data()[b] > es.size())
        throw std::invalid_argument("demux_batch: segment out of bounds");
    const uint8_t* p = buf.data();
    const int64_t* o = off.data();
    const int64_t* l = len.data();
    const int64_t* eo = es_off.data();
    int64_t total = 0;
    for (int64_t b = 0; b < B; ++b) total += l[b];
    py::gil_scoped_release nogil;
    parallel_for(B, [&](int64_t b) {
      ts::demux_segment(p + o[b], l[b], e + eo[b], pp + b * ts::kClasses * max_pes * 3, max_pes,
                        ip + b * ts::kInfoWords);
    }, total);
  });
  m.def("mpeg_crc32", [](Arr<uint8_t> data) { return ts::mpeg_crc32(data.data(), static_cast<size_t>(data.size())); });
  m.attr("TS_INFO_WORDS") = ts::kInfoWords;
  m.attr("TS_CLASSES") = ts::kClasses;

  // ------------------------------------------------------------------ store
  m.def("key_digest", [](Arr<int64_t> keys) {
    // int64[n, 4] segment keys -> uint32[n]: the digest a keyed CRC is bound with
    if (keys.size() % 4) throw std::invalid_argument("key_digest: keys must be int64[n, 4]");
    const int64_t n = keys.size() / 4;
    Arr<uint32_t> out(n);
    for (int64_t i = 0; i < n; ++i) out.mutable_data()[i] = key_digest(key_from(keys.data() + 4 * i));
    return out;
  });
  py::class_<SegmentStore>(m, "SegmentStore")
      .def(py::init<int64_t, int64_t>(), py::arg("capacity"), py::arg("align") = 256)
      .def_property_readonly("capacity", &SegmentStore::capacity)
      .def_property_readonly("used_bytes", &SegmentStore::used_bytes)
      .def_property_readonly("num_entries", &SegmentStore::num_entries)
      .def_property_readonly("evictions", &SegmentStore::evictions)
      .def_property_readonly("max_entries", &SegmentStore::max_entries)
      .def("lookup", [](const SegmentStore& s, Arr<int64_t> keys, bool include_pending) {
        const int64_t n = keys.size() / 4;
        Arr<int64_t> out(n);
        const int64_t* k = keys.data();
        int64_t* o = out.mutable_data();
        for (int64_t i = 0; i < n; ++i) o[i] = s.lookup(key_from(k + 4 * i), include_pending);
        return out;
      }, py::arg("keys"), py::arg("include_pending") = false)
      .def("lookup1", [](const SegmentStore& s, uint32_t swarm, uint32_t level, uint32_t url_id, uint32_t sn) {
        return s.lookup(SegKey{swarm, level, url_id, sn}, false);
      })
      .def("entries", [](const SegmentStore& s, Arr<int64_t> ids) {
        // -> int64[n, 4]: offset, length, state, pins
        const int64_t n = ids.size();
        Arr<int64_t> out({n, int64_t(4)});
        int64_t* o = out.mutable_data();
        for (int64_t i = 0; i < n; ++i) {
          int64_t id = ids.data()[i];
          if (id < 0 || id >= s.max_entries()) throw std::out_of_range("bad entry id");
          const Entry& e = s.entry(id);
          o[4 * i] = e.offset; o[4 * i + 1] = e.length; o[4 * i + 2] = e.state; o[4 * i + 3] = e.pins;
        }
        return out;
      })
      .def("reserve_run", [](SegmentStore& s, Arr<int64_t> keys, Arr<int64_t> lens, int64_t tick) -> py::object {
        const int64_t n = lens.size();
        if (keys.size() != 4 * n) throw std::invalid_argument("keys must be int64[n,4]");
        std::vector<SegKey> k(n);
        for (int64_t i = 0; i < n; ++i) k[i] = key_from(keys.data() + 4 * i);
        Arr<int64_t> ids(n), offs(n);
        int64_t base = s.reserve_run(k.data(), lens.data(), n, tick, ids.mutable_data(), offs.mutable_data());
        if (base < 0) return py::none();
        return py::make_tuple(base, ids, offs);
      })
      .def("p2p_layout", [](SegmentStore& s, Arr<int64_t> send_rows, Arr<int64_t> send_eids, Arr<int64_t> recv_rows,
                            int64_t tick) {
        // One round's P2P buffers (node.py:_p2p_phase), in one call.  Plan rows (sorted by
        // (src, dst, key)): [key x4, len, src, dst, want_id, seeded].
        //  sends, per destination run: (dst, row_a, row_b, mode, offset, total) -- mode 0:
        //    the run's entries lie back to back in the arena (aligned), send arena[offset,
        //    offset + total) as is; mode 1: gather into a staging buffer of `total` bytes,
        //    copies listed in `gathers` (run, arena offset, buffer offset, length).
        //  recvs, per source run: (src, row_a, row_b, base, total) -- one contiguous ring
        //    reservation, entries pinned; rid / roff: entry id / offset per recv row.
        const int64_t ns = send_eids.size();
        const int64_t nr = recv_rows.ndim() == 2 ? recv_rows.shape(0) : 0;
        if (ns && (send_rows.ndim() != 2 || send_rows.shape(0) != ns || send_rows.shape(1) < 9))
          throw std::invalid_argument("send_rows must be int64[n, >=9] aligned with send_eids");
        if (nr && recv_rows.shape(1) < 9) throw std::invalid_argument("recv_rows must be int64[n, >=9]");
        const int64_t sc = ns ? send_rows.shape(1) : 9, rc = nr ? recv_rows.shape(1) : 9;
        const int64_t* sr = send_rows.data();
        const int64_t* se = send_eids.data();
        const int64_t* rr = recv_rows.data();
        std::vector<int64_t> srun, gath;
        for (int64_t a = 0; a < ns;) {
          const int64_t dst = sr[a * sc + 6];
          int64_t b = a + 1;
          while (b < ns && sr[b * sc + 6] == dst) ++b;
          bool contiguous = true;
          int64_t total = 0;
          for (int64_t i = a; i < b && contiguous; ++i) {
            const int64_t id = se[i];
            if (id < 0 || id >= s.max_entries()) { contiguous = false; break; }
            const Entry& e = s.entry(id);
            if (e.length != sr[i * sc + 4]) contiguous = false;
            if (i > a) {
              const Entry& p = s.entry(se[i - 1]);
              if (e.offset != p.offset + s.aligned(p.length)) contiguous = false;
            }
          }
          if (contiguous) {
            const Entry& f = s.entry(se[a]);
            const Entry& l = s.entry(se[b - 1]);
            total = l.offset + l.length - f.offset;
            srun.insert(srun.end(), {dst, a, b, 0, f.offset, total});
          } else {
            const int64_t run = static_cast<int64_t>(srun.size() / 6);
            int64_t pos = 0;
            for (int64_t i = a; i < b; ++i) {
              const int64_t len = sr[i * sc + 4];
              const int64_t id = se[i];
              if (id >= 0 && id < s.max_entries()) {
                const Entry& e = s.entry(id);
                gath.insert(gath.end(), {run, e.offset, pos, std::min(e.length, len)});
              }
              total = pos + len;
              pos += s.aligned(len);
            }
            srun.insert(srun.end(), {dst, a, b, 1, -1, total});
          }
          a = b;
        }
        std::vector<int64_t> rrun;
        Arr<int64_t> rid(nr), roff(nr);
        for (int64_t a = 0; a < nr;) {
          const int64_t src = rr[a * rc + 5];
          int64_t b = a + 1;
          while (b < nr && rr[b * rc + 5] == src) ++b;
          const int64_t n = b - a;
          std::vector<SegKey> keys(n);
          std::vector<int64_t> lens(n);
          for (int64_t i = 0; i < n; ++i) {
            keys[i] = key_from(rr + (a + i) * rc);
            lens[i] = rr[(a + i) * rc + 4];
          }
          const int64_t base = s.reserve_run(keys.data(), lens.data(), n, tick, rid.mutable_data() + a,
                                             roff.mutable_data() + a);
          if (base < 0) throw std::runtime_error("segment cache cannot make room for peer data");
          for (int64_t i = a; i < b; ++i) s.pin(rid.data()[i]);
          const int64_t total = roff.data()[b - 1] + lens[n - 1] - roff.data()[a];
          rrun.insert(rrun.end(), {src, a, b, roff.data()[a], total});
          a = b;
        }
        auto as2d = [](const std::vector<int64_t>& v, int64_t cols) {
          const int64_t rows = static_cast<int64_t>(v.size()) / cols;
          Arr<int64_t> out({rows, cols});
          if (rows) std::memcpy(out.mutable_data(), v.data(), v.size() * sizeof(int64_t));
          return out;
        };
        return py::make_tuple(as2d(srun, 6), as2d(gath, 4), as2d(rrun, 5), rid, roff);
      })
      .def("fits", &SegmentStore::fits)
      // ---- replicated-state audit (agent/audit.py)
      .def("audit", [](const SegmentStore& s) {
        std::vector<std::string> e;
        s.audit(&e);
        return e;
      })
      .def_property_readonly("unpin_underflows", &SegmentStore::unpin_underflows)
      .def("region_start", &SegmentStore::region_start)
      .def("pin_table", [](const SegmentStore& s) {
        // -> (ids int64[n], pins int64[n]) of live entries holding pins
        std::vector<int64_t> ids, pins;
        for (int64_t i = 0; i < s.max_entries(); ++i) {
          const Entry& e = s.entry(i);
          if (e.state != kFree && e.pins != 0) {
            ids.push_back(i);
            pins.push_back(e.pins);
          }
        }
        Arr<int64_t> a(static_cast<py::ssize_t>(ids.size())), b(static_cast<py::ssize_t>(pins.size()));
        if (!ids.empty()) {
          std::memcpy(a.mutable_data(), ids.data(), ids.size() * sizeof(int64_t));
          std::memcpy(b.mutable_data(), pins.data(), pins.size() * sizeof(int64_t));
        }
        return py::make_tuple(a, b);
      })
      .def("live_entries", [](const SegmentStore& s) {
        // -> int64[n, 9]: id, key x4, offset, alloc bytes, state, indexed (the index names it)
        std::vector<int64_t> rows;
        for (int64_t i = 0; i < s.max_entries(); ++i) {
          const Entry& e = s.entry(i);
          if (e.state == kFree) continue;
          const int64_t ix = s.lookup(e.key, true);
          rows.insert(rows.end(), {i, int64_t(e.key.swarm), int64_t(e.key.level), int64_t(e.key.url_id),
                                   int64_t(e.key.sn), e.offset, e.alloc_bytes, int64_t(e.state), ix == i ? 1 : 0});
        }
        const int64_t n = static_cast<int64_t>(rows.size() / 9);
        Arr<int64_t> out({n, int64_t(9)});
        if (n) std::memcpy(out.mutable_data(), rows.data(), rows.size() * sizeof(int64_t));
        return out;
      })
      .def("peek_delta", [](const SegmentStore& s) {
        // -> (added int64[n,4], removed int64[m,4]) not taken yet
        std::vector<SegKey> add, rm;
        s.peek_delta(&add, &rm);
        auto keys = [](const std::vector<SegKey>& v) {
          Arr<int64_t> a({int64_t(v.size()), int64_t(4)});
          int64_t* p = a.mutable_data();
          for (size_t i = 0; i < v.size(); ++i) {
            p[4 * i] = v[i].swarm; p[4 * i + 1] = v[i].level; p[4 * i + 2] = v[i].url_id; p[4 * i + 3] = v[i].sn;
          }
          return a;
        };
        return py::make_tuple(keys(add), keys(rm));
      })
      .def("wrap_for", &SegmentStore::wrap_for)
      .def("retire_region", &SegmentStore::retire_region)
      .def("resident", [](const SegmentStore& s) {
        // -> (ids int64[n], keys int64[n,4]) of resident entries, oldest first
        std::vector<int64_t> ids;
        s.resident_ids(&ids);
        const int64_t n = static_cast<int64_t>(ids.size());
        Arr<int64_t> id_arr(n), keys({n, int64_t(4)});
        int64_t* k = keys.mutable_data();
        for (int64_t i = 0; i < n; ++i) {
          id_arr.mutable_data()[i] = ids[i];
          const SegKey& key = s.entry(ids[i]).key;
          k[4 * i] = key.swarm; k[4 * i + 1] = key.level; k[4 * i + 2] = key.url_id; k[4 * i + 3] = key.sn;
        }
        return py::make_tuple(id_arr, keys);
      })
      .def("aligned", &SegmentStore::aligned)
      .def("commit", [](SegmentStore& s, Arr<int64_t> ids) {
        for (int64_t i = 0; i < ids.size(); ++i) s.commit(ids.data()[i]);
      })
      .def("drop", [](SegmentStore& s, Arr<int64_t> ids) {
        for (int64_t i = 0; i < ids.size(); ++i) s.drop(ids.data()[i]);
      })
      .def("pin", [](SegmentStore& s, Arr<int64_t> ids) {
        for (int64_t i = 0; i < ids.size(); ++i) s.pin(ids.data()[i]);
      })
      .def("detach", [](SegmentStore& s, Arr<int64_t> ids) {
        for (int64_t i = 0; i < ids.size(); ++i) s.detach(ids.data()[i]);
      })
      .def("unpin", [](SegmentStore& s, Arr<int64_t> ids) {
        for (int64_t i = 0; i < ids.size(); ++i) s.unpin(ids.data()[i]);
      })
      .def("evict_below", &SegmentStore::evict_below)
      .def("take_delta", [](SegmentStore& s) {
        std::vector<SegKey> add, rm;
        std::vector<int64_t> add_len;
        s.take_delta(&add, &add_len, &rm);
        Arr<int64_t> a({int64_t(add.size()), int64_t(5)}), r({int64_t(rm.size()), int64_t(4)});
        int64_t* ap = a.mutable_data();
        for (size_t i = 0; i < add.size(); ++i) {
          ap[5 * i] = add[i].swarm; ap[5 * i + 1] = add[i].level; ap[5 * i + 2] = add[i].url_id;
          ap[5 * i + 3] = add[i].sn; ap[5 * i + 4] = add_len[i];
        }
        int64_t* rp = r.mutable_data();
        for (size_t i = 0; i < rm.size(); ++i) {
          rp[4 * i] = rm[i].swarm; rp[4 * i + 1] = rm[i].level; rp[4 * i + 2] = rm[i].url_id; rp[4 * i + 3] = rm[i].sn;
        }
        return py::make_tuple(a, r);
      });

  // ------------------------------------------------------------------ directory / planner
  py::class_<Directory>(m, "Directory")
      .def(py::init<>())
      .def_property_readonly("size", &Directory::size)
      // the content digest as a signed 64-bit word (it travels in an int64 control header)
      .def_property_readonly("digest", [](const Directory& d) { return static_cast<int64_t>(d.digest()); })
      .def("apply", [](Directory& d, int rank, Arr<int64_t> adds, Arr<int64_t> removes) {
        // adds int64[n,5] (key4, len); removes int64[m,4]
        for (int64_t i = 0; i < adds.size() / 5; ++i) d.apply_add(rank, key_from(adds.data() + 5 * i), adds.data()[5 * i + 4]);
        for (int64_t i = 0; i < removes.size() / 4; ++i) d.apply_remove(rank, key_from(removes.data() + 4 * i));
      })
      .def("drop_rank", &Directory::drop_rank)
      .def("holder_keys", [](const Directory& d, int rank) {
        // -> int64[n, 5]: key x4, length of the entries `rank` holds
        std::vector<SegKey> k;
        std::vector<int64_t> l;
        d.holder_keys(rank, &k, &l);
        Arr<int64_t> out({int64_t(k.size()), int64_t(5)});
        int64_t* p = out.mutable_data();
        for (size_t i = 0; i < k.size(); ++i) {
          p[5 * i] = k[i].swarm; p[5 * i + 1] = k[i].level; p[5 * i + 2] = k[i].url_id; p[5 * i + 3] = k[i].sn;
          p[5 * i + 4] = l[i];
        }
        return out;
      })
      .def("holders", [](const Directory& d, uint32_t swarm, uint32_t level, uint32_t url_id, uint32_t sn) {
        const DirEntry* e = d.find(SegKey{swarm, level, url_id, sn});
        return e ? e->holders : uint64_t(0);
      });
  // One round's gathered control messages (agent/node.py:_encode layout: header[hdr_words] =
  // magic, flags, #wants, #adds, #removes, leaving, round, cdn, p2p, upload, ...; then wants
  // [key4, size, want_id | force_cdn << 62 | not_staged << 61 | staging << 60 | held << 59], adds [key4, len], removes
  // [key4]) in one call:
  // applies every rank's cache delta to the directory and returns (want rows int64[n, 8] for
  // plan_round, per-rank flags, all-leaving, swarm byte totals [cdn, p2p, upload]).
  //
  // check_word >= 0: header words [check_word, check_word + 3) carry each rank's directory
  // digest taken before this ingest, the digest of the previous round's full plan and that
  // round's number.  They must agree on every rank: otherwise SwarmDivergence is raised
  // before anything is applied, naming the ranks behind each value, so no rank goes on to
  // post a send / receive group its peers do not match (a hang on a two-sided transport).
  m.def("ingest_control", [](Directory& d, const std::vector<Arr<int64_t>>& parts, int64_t magic,
                             int64_t hdr_words, int64_t check_word) {
    const int world = static_cast<int>(parts.size());
    Arr<int64_t> flags(world);
    int64_t tot[3] = {0, 0, 0};
    bool all_leaving = true;
    // pass 1: validate every header (nothing is applied from a round with a bad message) and
    // size the output; pass 2: apply the deltas and write the want rows straight into it
    int64_t n = 0;
    for (int r = 0; r < world; ++r) {
      const int64_t* p = parts[r].data();
      const int64_t size = parts[r].size();
      if (size < hdr_words || p[0] != magic) throw std::runtime_error("bad swarm control message");
      const int64_t nw = p[2], na = p[3], nr = p[4];
      if (nw < 0 || na < 0 || nr < 0 || hdr_words + 6 * nw + 5 * na + 4 * nr > size)
        throw std::runtime_error("truncated swarm control message");
      n += nw;
    }
    if (check_word >= 0 && check_word + 3 <= hdr_words && world > 1) {
      const int64_t* p0 = parts[0].data();
      for (int r = 1; r < world; ++r) {
        const int64_t* p = parts[r].data();
        if (p[check_word] != p0[check_word]) {
          std::ostringstream o;
          o << "swarm directory diverged before round " << p0[6] << " (replica digests "
            << group_ranks(parts, check_word) << ")";
          throw SwarmDivergence(o.str());
        }
        if (p[check_word + 1] != p0[check_word + 1] || p[check_word + 2] != p0[check_word + 2]) {
          std::ostringstream o;
          o << "swarm plans diverged in round " << p0[check_word + 2] << " (plan digests "
            << group_ranks(parts, check_word + 1) << "; planned rounds " << group_ranks(parts, check_word + 2)
            << ")";
          throw SwarmDivergence(o.str());
        }
      }
    }
    Arr<int64_t> out({n, int64_t(8)});
    int64_t* o = out.mutable_data();
    for (int r = 0; r < world; ++r) {
      const int64_t* p = parts[r].data();
      const int64_t nw = p[2], na = p[3], nr = p[4];
      flags.mutable_data()[r] = p[1];
      all_leaving = all_leaving && p[5] != 0;
      tot[0] += p[7];
      tot[1] += p[8];
      tot[2] += p[9];
      const int64_t* w = p + hdr_words;
      const int64_t* a = w + 6 * nw;
      const int64_t* rm = a + 5 * na;
      for (int64_t i = 0; i < na; ++i) d.apply_add(r, key_from(a + 5 * i), a[5 * i + 4]);
      for (int64_t i = 0; i < nr; ++i) d.apply_remove(r, key_from(rm + 4 * i));
      for (int64_t i = 0; i < nw; ++i, o += 8) {
        const int64_t* x = w + 6 * i;
        // want word: want_id | force_cdn << 62 | not_staged << 61 | staging << 60 | held << 59
        // -> WantFlag bits
        o[0] = x[0];
        o[1] = x[1];
        o[2] = x[2];
        o[3] = x[3];
        o[4] = x[4];
        o[5] = x[5] & ((int64_t(1) << 59) - 1);
        o[6] = r;
        o[7] = ((x[5] >> 62) & 1 ? kForceCdn : 0) | ((x[5] >> 61) & 1 ? kNotStaged : 0) |
               ((x[5] >> 60) & 1 ? kStaging : 0) | ((x[5] >> 59) & 1 ? kHeld : 0);
      }
    }
    Arr<int64_t> totals(3);
    std::memcpy(totals.mutable_data(), tot, sizeof(tot));
    return py::make_tuple(out, flags, all_leaving, totals);
  }, py::arg("directory"), py::arg("parts"), py::arg("magic"), py::arg("hdr_words"), py::arg("check_word") = -1);
  // wants: int64[n, 8] = (key4, size, want_id, rank, want_flags); flags int64[world]
  // -> int64[m, 10] = (key4, size, src, dst, want_id, seeded, reserved); src -1 = CDN fetch,
  // -2 = stage (download from a network origin into host memory for a later round)
  // plan_round_for: the same plan, but only the rows this rank takes part in (src == me or
  // dst == me, canonical order kept) plus whether the round has any P2P transfer at all
  // (every rank enters the exchange then) and the 64-bit digest of the full plan (ranks
  // compare it in the next round's control all-gather, see ingest_control).  At 8 ranks a
  // rank needs ~1/4 of the rows: the rest would be built into numpy and masked away in
  // Python every round.
  auto plan_rows = [](const Directory& d, const Arr<int64_t>& wants, const Arr<int64_t>& flags, int world,
                      int me, const py::object& cdn_obj) {
    const int64_t n = wants.size() / 8;
    if (flags.size() != world) throw std::invalid_argument("flags must have world entries");
    std::vector<Want> w(n);
    std::vector<Transfer> t;
    std::vector<int64_t> f;
    const int64_t* p = wants.data();
    for (int64_t i = 0; i < n; ++i) {
      w[i].key = key_from(p + 8 * i);
      w[i].size = p[8 * i + 4];
      w[i].want_id = p[8 * i + 5];
      w[i].rank = static_cast<int32_t>(p[8 * i + 6]);
      w[i].flags = p[8 * i + 7];
      if (w[i].rank < 0 || w[i].rank >= world) throw std::invalid_argument("want rank out of range");
    }
    f.assign(flags.data(), flags.data() + world);
    std::vector<int64_t> cdn;
    if (!cdn_obj.is_none()) {  // each rank's cumulative CDN bytes: the planner's CDN balance
      Arr<int64_t> c = cdn_obj.cast<Arr<int64_t>>();
      if (c.size() != world) throw std::invalid_argument("cdn_bytes must have world entries");
      cdn.assign(c.data(), c.data() + world);
    }
    plan_round_into(d, w.data(), w.size(), f, world, &t, cdn.empty() ? nullptr : cdn.data());
    const int64_t digest = static_cast<int64_t>(plan_digest(t));  // of the FULL plan, before filtering
    bool any_p2p = false;
    int64_t m = 0;
    for (const Transfer& x : t) {
      any_p2p = any_p2p || x.src >= 0;
      if (me < 0 || x.src == me || x.dst == me) ++m;
    }
    Arr<int64_t> out({m, int64_t(10)});
    int64_t* o = out.mutable_data();
    for (const Transfer& x : t) {
      if (me >= 0 && x.src != me && x.dst != me) continue;
      o[0] = x.key.swarm; o[1] = x.key.level; o[2] = x.key.url_id; o[3] = x.key.sn;
      o[4] = x.size; o[5] = x.src; o[6] = x.dst; o[7] = x.want_id; o[8] = x.seeded; o[9] = 0;
      o += 10;
    }
    return std::make_tuple(out, any_p2p, digest);
  };
  m.def("plan_round", [plan_rows](const Directory& d, Arr<int64_t> wants, Arr<int64_t> flags, int world,
                                  py::object cdn_bytes) {
    return std::get<0>(plan_rows(d, wants, flags, world, -1, cdn_bytes));
  }, py::arg("directory"), py::arg("wants"), py::arg("flags"), py::arg("world"), py::arg("cdn_bytes") = py::none());
  m.def("plan_round_for", [plan_rows](const Directory& d, Arr<int64_t> wants, Arr<int64_t> flags, int world,
                                      int me, py::object cdn_bytes) {
    if (me < 0 || me >= world) throw std::invalid_argument("rank out of range");
    auto r = plan_rows(d, wants, flags, world, me, cdn_bytes);
    return py::make_tuple(std::get<0>(r), std::get<1>(r), std::get<2>(r));
  }, py::arg("directory"), py::arg("wants"), py::arg("flags"), py::arg("world"), py::arg("me"),
     py::arg("cdn_bytes") = py::none());
  // CPU-mode CDN phase: copy origin byte ranges (raw host addresses, as the want table holds
  // them) into the node's host arena at `dst_base + dst_off[i]` (bounds-checked against cap)
  m.def("host_copy_batch", [](int64_t dst_base, int64_t dst_cap, Arr<int64_t> dst_off, Arr<int64_t> src_ptr,
                              Arr<int64_t> len) {
    const int64_t n = len.size();
    if (dst_off.size() != n || src_ptr.size() != n) throw std::invalid_argument("host_copy_batch: sizes differ");
    for (int64_t i = 0; i < n; ++i) {
      const int64_t o = dst_off.data()[i], l = len.data()[i];
      if (o < 0 || l < 0 || o + l > dst_cap) throw std::out_of_range("host_copy_batch: destination out of bounds");
      if (l && src_ptr.data()[i] == 0) throw std::invalid_argument("host_copy_batch: null source");
      if (l) std::memcpy(reinterpret_cast<uint8_t*>(dst_base) + o, reinterpret_cast<const uint8_t*>(src_ptr.data()[i]),
                         static_cast<size_t>(l));
    }
  });

  // ------------------------------------------------------------------ want table
  // (agent/node.py: the rank's per-request state as rows; see wants.hpp)
  py::class_<SegmentLocator>(m, "SegmentLocator")
      .def(py::init<>())
      .def("add_dir",
           [](SegmentLocator& l, const std::string& dir, const std::string& prefix, const std::string& suffix,
              int64_t sn_lo, int64_t sn_hi, int64_t base, int64_t flags, Arr<int64_t> off, Arr<int64_t> len) {
             if (off.size() != len.size()) throw std::invalid_argument("add_dir: off / len sizes differ");
             SegmentLocator::Dir d;
             d.prefix = prefix;
             d.suffix = suffix;
             d.sn_lo = sn_lo;
             d.sn_hi = sn_hi;
             d.base = base;
             d.flags = flags;
             d.off.assign(off.data(), off.data() + off.size());
             d.len.assign(len.data(), len.data() + len.size());
             l.add_dir(dir, std::move(d));
           },
           py::arg("dir"), py::arg("prefix"), py::arg("suffix"), py::arg("sn_lo"), py::arg("sn_hi"), py::arg("base"),
           py::arg("flags"), py::arg("off"), py::arg("len"))
      .def("resolve",
           [](const SegmentLocator& l, const py::list& urls) {
             // string views into the list's str objects (the GIL stays held: no other thread
             // can drop an item of the list while the views are in use)
             const size_t n = urls.size();
             std::vector<std::string_view> v(n);
             for (size_t i = 0; i < n; ++i) {
               Py_ssize_t len = 0;
               const char* s = PyUnicode_AsUTF8AndSize(urls[i].ptr(), &len);
               if (s == nullptr) throw py::error_already_set();
               v[i] = std::string_view(s, static_cast<size_t>(len));
             }
             py::array_t<int64_t> size(n), ptr(n), base(n), flags(n);
             py::array_t<uint8_t> ok(n);
             const int64_t found = l.resolve(v, size.mutable_data(), ptr.mutable_data(), base.mutable_data(),
                                             flags.mutable_data(), ok.mutable_data());
             return py::make_tuple(size, ptr, base, flags, ok.attr("astype")("bool"), found);
           })
      .def("clear", &SegmentLocator::clear)
      .def("__len__", &SegmentLocator::size);

  py::class_<WantTable>(m, "WantTable")
      .def(py::init<>())
      .def("__len__", &WantTable::size)
      .def_property_readonly("waiting", &WantTable::waiting)
      .def_property_readonly("num_tokens", &WantTable::tokens)
      .def("add", [](WantTable& t, Arr<int64_t> keys, Arr<int64_t> sizes, Arr<int64_t> ptr, Arr<int64_t> base,
                     Arr<int64_t> flags, Arr<int64_t> tokens) {
        // -> (want ids int64[n], created uint8[n])
        const int64_t n = tokens.size();
        if (keys.size() != 4 * n || sizes.size() != n || ptr.size() != n || base.size() != n || flags.size() != n)
          throw std::invalid_argument("WantTable.add: keys int64[n,4] and n-long columns");
        Arr<int64_t> ids(n);
        Arr<uint8_t> created(n);
        const int64_t* k = keys.data();
        for (int64_t i = 0; i < n; ++i) {
          bool c = false;
          ids.mutable_data()[i] = t.add(key_from(k + 4 * i), sizes.data()[i], ptr.data()[i], base.data()[i],
                                        static_cast<int32_t>(flags.data()[i]), tokens.data()[i], &c);
          created.mutable_data()[i] = c ? 1 : 0;
        }
        return py::make_tuple(ids, created);
      })
      .def("add1", [](WantTable& t, uint32_t swarm, uint32_t level, uint32_t url_id, uint32_t sn, int64_t size,
                      int64_t ptr, int64_t base, int64_t flags, int64_t token) {
        // -> want id, negated - 1 when the want was created (one int back, no tuple)
        bool c = false;
        const int64_t id = t.add(SegKey{swarm, level, url_id, sn}, size, ptr, base, static_cast<int32_t>(flags),
                                 token, &c);
        return c ? -id - 1 : id;
      })
      .def("abort", [](WantTable& t, Arr<int64_t> tokens) {
        int64_t n = 0;
        for (int64_t i = 0; i < tokens.size(); ++i) n += t.abort(tokens.data()[i]) ? 1 : 0;
        return n;
      })
      .def("abort1", &WantTable::abort)
      .def("lookup1", [](const WantTable& t, uint32_t swarm, uint32_t level, uint32_t url_id, uint32_t sn) {
        return t.lookup(SegKey{swarm, level, url_id, sn});
      })
      .def("select", [](WantTable& t, const SegmentStore& store, const Directory* dir, int64_t cap, int32_t round) {
        // -> (admitted ids, control rows int64[k, 6], dropped ids, too-big ids, deferred count)
        std::vector<int64_t> adm, dropped, big;
        int64_t deferred = 0;
        t.select(store, dir, cap, round, &adm, &dropped, &big, &deferred);
        const int64_t k = static_cast<int64_t>(adm.size());
        Arr<int64_t> rows({k, int64_t(6)});
        if (k) t.encode(adm.data(), k, rows.mutable_data());
        auto vec = [](const std::vector<int64_t>& v) {
          Arr<int64_t> a(static_cast<py::ssize_t>(v.size()));
          if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(int64_t));
          return a;
        };
        return py::make_tuple(vec(adm), rows, vec(dropped), vec(big), deferred);
      }, py::arg("store"), py::arg("directory").none(true), py::arg("cap"), py::arg("round"))
      .def("info", [](const WantTable& t, Arr<int64_t> ids) {
        // -> int64[n, 10]: key x4, size, src_ptr, src_base, flags, round, attempts (row of -1: unknown id)
        const int64_t n = ids.size();
        Arr<int64_t> out({n, int64_t(10)});
        int64_t* o = out.mutable_data();
        for (int64_t i = 0; i < n; ++i, o += 10) {
          const WantRec* r = t.get(ids.data()[i]);
          if (r == nullptr) {
            std::fill(o, o + 10, -1);
            continue;
          }
          o[0] = r->key.swarm; o[1] = r->key.level; o[2] = r->key.url_id; o[3] = r->key.sn;
          o[4] = r->size; o[5] = r->src_ptr; o[6] = r->src_base; o[7] = r->flags; o[8] = r->round;
          o[9] = r->attempts;
        }
        return out;
      })
      .def("set", [](WantTable& t, int64_t id, int64_t size, int64_t set_flags, int64_t clear_flags) {
        // size < 0: unchanged; returns False for an unknown id
        WantRec* r = t.get(id);
        if (r == nullptr) return false;
        if (size >= 0) r->size = size;
        r->flags = static_cast<int32_t>((r->flags | set_flags) & ~clear_flags);
        return true;
      }, py::arg("id"), py::arg("size") = -1, py::arg("set_flags") = 0, py::arg("clear_flags") = 0)
      .def("waiters", [](const WantTable& t, int64_t id) {
        const WantRec* r = t.get(id);
        std::vector<int64_t> w;
        if (r != nullptr) w = r->waiters;
        return w;
      })
      .def("finish", [](WantTable& t, Arr<int64_t> ids) {
        // -> (tokens int64[m], index of each token's want in ids int64[m], prefetch-only uint8[n])
        std::vector<int64_t> tok, idx;
        std::vector<uint8_t> pf;
        t.finish(ids.data(), ids.size(), &tok, &idx, &pf);
        Arr<int64_t> a(static_cast<py::ssize_t>(tok.size())), b(static_cast<py::ssize_t>(idx.size()));
        Arr<uint8_t> c(static_cast<py::ssize_t>(pf.size()));
        if (!tok.empty()) std::memcpy(a.mutable_data(), tok.data(), tok.size() * sizeof(int64_t));
        if (!idx.empty()) std::memcpy(b.mutable_data(), idx.data(), idx.size() * sizeof(int64_t));
        if (!pf.empty()) std::memcpy(c.mutable_data(), pf.data(), pf.size());
        return py::make_tuple(a, b, c);
      })
      .def("requeue", [](WantTable& t, Arr<int64_t> ids, bool force_cdn) { t.requeue(ids.data(), ids.size(), force_cdn); },
           py::arg("ids"), py::arg("force_cdn") = false)
      .def("audit", [](const WantTable& t) {
        std::vector<std::string> e;
        t.audit(&e);
        return e;
      })
      .def("ids", [](const WantTable& t) {
        std::vector<int64_t> v;
        t.ids(&v);
        Arr<int64_t> a(static_cast<py::ssize_t>(v.size()));
        if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(int64_t));
        return a;
      })
      .def("token_map", [](const WantTable& t) {
        // -> (tokens int64[n], want ids int64[n])
        std::vector<int64_t> tk, w;
        t.token_map(&tk, &w);
        Arr<int64_t> a(static_cast<py::ssize_t>(tk.size())), b(static_cast<py::ssize_t>(w.size()));
        if (!tk.empty()) {
          std::memcpy(a.mutable_data(), tk.data(), tk.size() * sizeof(int64_t));
          std::memcpy(b.mutable_data(), w.data(), w.size() * sizeof(int64_t));
        }
        return py::make_tuple(a, b);
      });
  m.attr("WANT_FORCE_CDN") = int64_t(kWForceCdn);
  m.attr("WANT_NOT_STAGED") = int64_t(kWNotStaged);
  m.attr("WANT_STAGING") = int64_t(kWStaging);
  m.attr("WANT_PREFETCH") = int64_t(kWPrefetch);
  m.attr("WANT_PY") = int64_t(kWPy);
  m.attr("WANT_CORRUPT") = int64_t(kWCorrupt);
  m.attr("WANT_HELD") = int64_t(kWHeld);
  m.attr("WANT_ON_DEV") = int64_t(kWOnDev);
  m.attr("NO_TOKEN") = kNoToken;

  // ------------------------------------------------------------------ intra-node control plane
  py::class_<ShmControl>(m, "ShmControl")
      .def(py::init<const std::string&, int, int, int64_t, bool>(), py::arg("name"), py::arg("rank"),
           py::arg("world"), py::arg("slot_words"), py::arg("create"))
      .def("unlink", &ShmControl::unlink)
      .def_property_readonly("slot_words", &ShmControl::slot_words)
      .def_property_readonly("generation", &ShmControl::generation)
      // all-gather of int64 vectors; None when some rank's message exceeded slot_words
      // (every rank sees the same lengths, so all of them take the caller's fallback)
      .def("allgather",
           [](ShmControl& s, Arr<int64_t> msg, double timeout_s) -> py::object {
             const int64_t n = msg.size();
             {
               py::gil_scoped_release nogil;
               s.exchange(msg.data(), n, timeout_s);
             }
             std::vector<int64_t> lens(s.world());
             for (int r = 0; r < s.world(); ++r) {
               lens[r] = s.length(r);
               if (lens[r] > s.slot_words()) return py::none();
             }
             py::list out;
             for (int r = 0; r < s.world(); ++r) {
               Arr<int64_t> a(static_cast<py::ssize_t>(lens[r]));
               s.read(r, a.mutable_data());
               out.append(a);
             }
             return std::move(out);
           },
           py::arg("msg"), py::arg("timeout_s") = 300.0)
      .def("barrier", [](ShmControl& s, double timeout_s) {
        py::gil_scoped_release nogil;
        s.barrier(timeout_s);
      }, py::arg("timeout_s") = 300.0);

  m.attr("FLAG_ONLINE") = int64_t(kOnline);
  m.attr("FLAG_UPLOAD") = int64_t(kUploadOn);
  m.attr("FLAG_DOWNLOAD") = int64_t(kDownloadOn);
  m.attr("FLAG_CDN_DEDUP") = int64_t(kCdnDedup);
  m.attr("FLAG_CDN_BOUND") = int64_t(kCdnBound);
}
