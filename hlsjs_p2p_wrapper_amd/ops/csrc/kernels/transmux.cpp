// One native call per transmux batch (player/transmux.py, SURVEY §2.2 K10 + K11): the
// per-segment descriptor math of AES-128-CBC decrypt and MPEG-TS demux, ONE pinned staging
// block + ONE H2D for every descriptor of the batch, the decrypt launch, the demux launch
// sequence per group (encrypted segments demux from the decrypt buffer with their plaintext
// lengths read on device; clear ones in place), and the async D2H of the small per-segment
// info rows and plaintext lengths into one pinned block.
//
// The same steps in Python (ops/aes.py + ops/tsdemux.py: numpy prefix sums, two descriptor
// packs, argument checks, six pybind launches, two pinned allocations) cost ~0.2 ms of host
// time per 64-segment batch -- the host path bounds the per-GPU segment rate once peers
// share the CDN work (N > 1); here it is tens of microseconds.
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>
#include <torch/extension.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace hlsp2p {
namespace dev {
int aes_chunk_blocks();
hipError_t launch_aes128_cbc_decrypt(const uint8_t*, uint8_t*, const int64_t*, const int64_t*, const int64_t*,
                                     const int64_t*, const uint32_t*, const uint32_t*, const uint32_t*,
                                     const uint8_t*, int64_t*, int, int64_t, int, hipStream_t, const int64_t*,
                                     const void*, uint32_t*, const int64_t*, void*);
hipError_t launch_ts_demux(const uint8_t*, const int64_t*, const int64_t*, const int64_t*, int, int64_t, uint32_t*,
                           int64_t*, int32_t*, uint8_t*, const int64_t*, int64_t*, int64_t, int64_t*, hipStream_t,
                           const void*, const int64_t*);
hipError_t launch_crc32_from_masks(const uint32_t*, const void*, const int64_t*, const int64_t*, const uint32_t*, uint32_t*, uint32_t*,
                                   const uint32_t*, uint8_t*, const int64_t*, uint32_t*, int64_t, int, int64_t, int,
                                   hipStream_t);
}  // namespace dev
}  // namespace hlsp2p

namespace {

namespace py = pybind11;
using torch::Tensor;
using I64 = py::array_t<int64_t, py::array::c_style | py::array::forcecast>;

constexpr int64_t kAlign = 256;   // segment start alignment in the decrypt / ES buffers
constexpr int64_t kPacket = 188;  // MPEG-TS packet
constexpr int64_t kInfo = 24;     // int64 words per segment info row (ops/tsdemux.py INFO_WORDS)

int64_t align_up(int64_t n) { return (n + kAlign - 1) / kAlign * kAlign; }

// host time of transmux_launch by stage (transmux_launch_profile): checks + plans,
// descriptor upload, result allocations, decrypt (+ fused CRC) launches, demux launches + D2H
// copies, Python results; with the call count.  Plain globals: every call holds the GIL (the
// binding never releases it), so calls from several Python threads are serialized
enum { kStPlan, kStDesc, kStAlloc, kStDecrypt, kStDemux, kStResult, kStDescPin, kStDescCopy, kStDescDev, kStDescH2D,
       kStages };
std::array<double, kStages> g_stage_us{};
int64_t g_calls = 0;
using Clock = std::chrono::steady_clock;
struct StageClock {
  Clock::time_point t = Clock::now();
  void lap(int stage) {
    const auto now = Clock::now();
    g_stage_us[stage] += std::chrono::duration<double, std::micro>(now - t).count();
    t = now;
  }
};

// Host staging of many small arrays, 16-byte aligned, copied to the device in one H2D.
class Desc {
 public:
  int64_t add(const void* p, int64_t nbytes) {
    const int64_t off = static_cast<int64_t>(buf_.size());
    buf_.resize(off + ((nbytes + 15) & ~int64_t(15)), 0);
    if (nbytes) std::memcpy(buf_.data() + off, p, static_cast<size_t>(nbytes));
    return off;
  }
  template <typename T>
  int64_t add(const std::vector<T>& v) { return add(v.data(), static_cast<int64_t>(v.size() * sizeof(T))); }
  // pinned block from the caching host allocator (recorded on the copy's stream, so reuse
  // waits for the copy), one non-blocking H2D on the current stream
  Tensor upload(int device, StageClock& clk) {
    const int64_t n = std::max<int64_t>(16, static_cast<int64_t>(buf_.size()));
    clk.lap(kStDesc);
    Tensor host = torch::empty({n}, torch::TensorOptions().dtype(torch::kUInt8).pinned_memory(true));
    clk.lap(kStDescPin);
    std::memcpy(host.data_ptr<uint8_t>(), buf_.data(), buf_.size());
    clk.lap(kStDescCopy);
    Tensor d = torch::empty({n}, torch::TensorOptions().dtype(torch::kUInt8).device(torch::kCUDA, device));
    clk.lap(kStDescDev);
    d.copy_(host, /*non_blocking=*/true);
    clk.lap(kStDescH2D);
    dev_ = d;
    return d;
  }
  template <typename T>
  T* at(int64_t off) const { return reinterpret_cast<T*>(static_cast<uint8_t*>(dev_.data_ptr()) + off); }
  Tensor device() const { return dev_; }

 private:
  std::vector<uint8_t> buf_;
  Tensor dev_;
};

struct DemuxPlan {
  std::vector<int64_t> idx, off, len, cap, es_off, es_cap, blk_prefix;
  int64_t es_bytes = 0, total_blocks = 0;
  int64_t d_off = -1, d_len = -1, d_bp = -1, d_eo = -1;
};

void plan_demux(DemuxPlan& p) {
  const size_t B = p.idx.size();
  p.es_off.resize(B);
  p.es_cap.resize(B);
  p.blk_prefix.assign(B + 1, 0);
  int64_t pos = 0;
  for (size_t i = 0; i < B; ++i) {
    p.es_off[i] = pos;
    p.es_cap[i] = align_up(std::max<int64_t>(p.cap[i], 1));
    pos += p.es_cap[i];
    const int64_t blocks = ((p.cap[i] + kPacket - 1) / kPacket + 255) / 256;  // 256-packet demux blocks
    p.blk_prefix[i + 1] = p.blk_prefix[i] + blocks;
  }
  p.es_bytes = pos + kAlign;
  p.total_blocks = p.blk_prefix[B];
}

int cus(int device) {
  static int cached[64] = {0};
  if (device >= 0 && device < 64 && cached[device]) return cached[device];
  int n = 0;
  hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device);
  if (n <= 0) n = 256;
  if (device >= 0 && device < 64) cached[device] = n;
  return n;
}

// CUs the persistent decrypt grid leaves free (set_cu_reserve): with a live RCCL data plane
// the node stream's send/recv kernels must find a CU while a decrypt batch runs -- one
// 1024-thread AES workgroup with its 160 KiB LDS image fills a CU (waves, VGPRs and LDS), so
// a full-chip persistent grid would hold RCCL back for the whole batch.
int g_cu_reserve = 0;

// HLSP2P_DECRYPT_CUS: at most this many CUs for the decrypt grid -- the rest stay free for the
// memory-bound kernels of the other streams (ingest copies, CRC, the previous batch's demux):
// one 160 KiB decrypt workgroup fills a CU's LDS, so nothing that needs LDS co-resides with it
int g_decrypt_cap = -1;
int decrypt_cus(int device) {
  if (g_decrypt_cap < 0) {
    const char* v = std::getenv("HLSP2P_DECRYPT_CUS");
    g_decrypt_cap = v != nullptr ? std::max(0, std::atoi(v)) : 0;
  }
  int n = cus(device) - g_cu_reserve;
  if (g_decrypt_cap > 0) n = std::min(n, g_decrypt_cap);
  return std::max(8, n);
}

void hip_ok(hipError_t e, const char* what) { TORCH_CHECK(e == hipSuccess, what, " failed: ", hipGetErrorString(e)); }

// src: uint8 device buffer holding every payload at src_off[i] (16-byte aligned) with
// nbytes[i] bytes; enc[i] != 0 -> AES-128-CBC with round keys drk[i] (44 little-endian
// words, equivalent inverse cipher) and IV iv[i]; encrypted sizes must be positive
// multiples of 16 (the caller rejects others).  Returns, per group (encrypted, then clear):
// (indices into the batch, info [B,24] device, pes device, es buffer, es offsets,
// info rows in pinned host memory, plaintext lengths in pinned host memory (enc) or a
// host array (clear)); plus the decrypt buffer to keep alive until the batch completes.
py::tuple transmux_launch(Tensor src, I64 src_off, I64 nbytes, py::array_t<uint8_t, py::array::c_style> enc,
                          py::array_t<uint32_t, py::array::c_style | py::array::forcecast> drk,
                          py::array_t<uint8_t, py::array::c_style | py::array::forcecast> iv, Tensor td0, Tensor isb,
                          int64_t max_pes, py::object expect_obj, c10::optional<Tensor> crc_w,
                          c10::optional<Tensor> crc_tables) {
  StageClock clk;
  ++g_calls;
  TORCH_CHECK_VALUE(src.is_cuda() && src.is_contiguous() && src.scalar_type() == torch::kUInt8, "src: contiguous GPU uint8");
  TORCH_CHECK_VALUE((reinterpret_cast<uintptr_t>(src.data_ptr()) & 15) == 0, "src must be 16-byte aligned");
  const int64_t B = src_off.size();
  TORCH_CHECK_VALUE(nbytes.size() == B && enc.size() == B, "transmux_launch: argument sizes differ");
  TORCH_CHECK_VALUE(drk.ndim() == 2 && drk.shape(0) == B && drk.shape(1) == 44, "drk must be [B, 44]");
  TORCH_CHECK_VALUE(iv.ndim() == 2 && iv.shape(0) == B && iv.shape(1) == 16, "iv must be [B, 16]");
  TORCH_CHECK_VALUE(td0.is_cuda() && td0.numel() >= 256 && isb.is_cuda() && isb.numel() >= 256, "AES tables");
  TORCH_CHECK_VALUE(max_pes > 0, "max_pes must be positive");
  const int64_t* so = src_off.data();
  const int64_t* nb = nbytes.data();
  const uint8_t* en = enc.data();
  const int64_t cap_src = src.numel();
  const int device = src.get_device();
  for (int64_t i = 0; i < B; ++i) {
    TORCH_CHECK_VALUE(so[i] >= 0 && nb[i] >= 0 && so[i] + nb[i] <= cap_src, "payload out of bounds");
    TORCH_CHECK_VALUE(so[i] % 16 == 0, "payload offsets must be 16-byte aligned");
    if (en[i]) {
      TORCH_CHECK_VALUE(nb[i] >= 16 && nb[i] % 16 == 0, "encrypted payload is not a positive multiple of 16");
      TORCH_CHECK_VALUE(nb[i] < (int64_t(1) << 31), "encrypted payload over 2 GiB (the decrypt's buffer ranges)");
    }
  }
  const auto dev_opts = torch::TensorOptions().device(torch::kCUDA, device);
  hipStream_t st = c10::hip::getCurrentHIPStream(device).stream();
  // optional verify: expect[i] >= 0 is the CRC-32 the CIPHERTEXT of encrypted segment i must
  // have (a peer's trailer); the decrypt computes it on the fly (aes_cbc.hip AesCrc)
  std::vector<int64_t> v_exp;
  if (!expect_obj.is_none()) {
    I64 ex = expect_obj.cast<I64>();
    TORCH_CHECK_VALUE(ex.size() == B, "expect must have one entry per segment");
    v_exp.assign(ex.data(), ex.data() + B);
    bool any = false;
    for (int64_t i = 0; i < B; ++i) {
      if (v_exp[i] < 0) continue;
      TORCH_CHECK_VALUE(en[i], "fused CRC verify needs an encrypted segment (verify clear ones separately)");
      any = true;
    }
    if (!any) v_exp.clear();
    else
      TORCH_CHECK_VALUE(crc_w.has_value() && crc_tables.has_value() && crc_w->is_cuda() &&
                            crc_w->numel() * crc_w->element_size() >= (8 + 32) * 64 * 16 && crc_tables->is_cuda() &&
                            crc_tables->numel() >= (40 + 12) * 1024,
                        "fused CRC verify needs the chunk weights and shift tables on the device");
  }

  // ---- plans: AES over the encrypted segments, demux per group
  std::vector<int64_t> a_so, a_do, a_bp{0}, a_cp{0};
  std::vector<int64_t> a_mo, v_idx, v_coff, v_len, v_expw;  // fused CRC: mask offsets, verify columns
  int64_t v_chunks = 0;
  // packet-header records for the demux scan, written by the decrypt (aes_cbc.hip AesHdr):
  // per encrypted segment nb / 188 + 2 16-byte records (HLSP2P_HDR_RECORDS=0: off, the scan
  // reads the plaintext)
  static const bool hdr_on = [] {
    const char* v = std::getenv("HLSP2P_HDR_RECORDS");
    return v == nullptr || std::strcmp(v, "0") != 0;
  }();
  std::vector<int64_t> a_ho;
  int64_t hdr_pos = 0;
  std::vector<uint32_t> a_drk;
  std::vector<uint8_t> a_iv;
  DemuxPlan pe, pc;
  const int64_t chunk = hlsp2p::dev::aes_chunk_blocks();
  int64_t dec_pos = 0;
  for (int64_t i = 0; i < B; ++i) {
    if (en[i]) {
      a_so.push_back(so[i]);
      a_do.push_back(dec_pos);
      pe.idx.push_back(i);
      pe.off.push_back(dec_pos);
      pe.cap.push_back(nb[i]);
      dec_pos += align_up(nb[i]);
      const int64_t blocks = nb[i] / 16;
      a_bp.push_back(a_bp.back() + blocks);
      a_cp.push_back(a_cp.back() + (blocks + chunk - 1) / chunk);
      a_ho.push_back(hdr_pos);
      hdr_pos += nb[i] / kPacket + 2;
      if (!v_exp.empty()) {
        const int64_t nch = (blocks + chunk - 1) / chunk;  // one 4096-byte CRC chunk per decrypt chunk
        if (v_exp[i] >= 0) {
          a_mo.push_back(64 * v_chunks);  // crc_host.hpp kFusedMaskDwords
          v_idx.push_back(i);
          v_coff.push_back(v_chunks);
          v_len.push_back(nb[i]);
          v_expw.push_back(v_exp[i] & 0xffffffffll);
          v_chunks += nch;
        } else {
          a_mo.push_back(-1);
        }
      }
      a_drk.insert(a_drk.end(), drk.data(i, 0), drk.data(i, 0) + 44);
      a_iv.insert(a_iv.end(), iv.data(i, 0), iv.data(i, 0) + 16);
    } else {
      pc.idx.push_back(i);
      pc.off.push_back(so[i]);
      pc.cap.push_back(nb[i]);
      pc.len.push_back(nb[i]);
    }
  }
  const int64_t ne = static_cast<int64_t>(pe.idx.size()), nc = static_cast<int64_t>(pc.idx.size());
  plan_demux(pe);
  plan_demux(pc);

  clk.lap(kStPlan);
  // ---- every descriptor of the batch in one staging block, one H2D
  Desc desc;
  int64_t d_so = -1, d_do = -1, d_bp = -1, d_cp = -1, d_drk = -1, d_iv = -1, d_mo = -1, d_vco = -1, d_vl = -1,
          d_vx = -1, d_ho = -1;
  const int64_t nv = static_cast<int64_t>(v_idx.size());
  if (ne) {
    d_so = desc.add(a_so);
    d_do = desc.add(a_do);
    d_bp = desc.add(a_bp);
    d_cp = desc.add(a_cp);
    d_drk = desc.add(a_drk);
    d_iv = desc.add(a_iv);
    pe.d_off = desc.add(pe.off);
    pe.d_bp = desc.add(pe.blk_prefix);
    pe.d_eo = desc.add(pe.es_off);
    if (hdr_on) d_ho = desc.add(a_ho);
    if (nv) {
      std::vector<uint32_t> ex32(v_expw.begin(), v_expw.end());
      d_mo = desc.add(a_mo);
      d_vco = desc.add(v_coff);
      d_vl = desc.add(v_len);
      d_vx = desc.add(ex32);
    }
  }
  if (nc) {
    pc.d_off = desc.add(pc.off);
    pc.d_len = desc.add(pc.len);
    pc.d_bp = desc.add(pc.blk_prefix);
    pc.d_eo = desc.add(pc.es_off);
  }
  desc.upload(device, clk);

  // ---- host results block: info rows (enc group, then clear group) | enc plaintext lengths
  Tensor host = torch::empty({(ne + nc) * kInfo + ne + 1}, torch::TensorOptions().dtype(torch::kInt64).pinned_memory(true));
  Tensor dec, out_len;
  if (ne) out_len = torch::empty({ne}, dev_opts.dtype(torch::kInt64));
  Tensor masks, chunk_res, v_crc, v_ok, v_ok_host;
  if (nv) {
    masks = torch::empty({64 * v_chunks}, dev_opts.dtype(torch::kInt32));
    chunk_res = torch::empty({std::max<int64_t>(1, v_chunks)}, dev_opts.dtype(torch::kInt32));
    v_crc = torch::empty({nv}, dev_opts.dtype(torch::kInt32));
    v_ok = torch::empty({nv}, dev_opts.dtype(torch::kUInt8));
  }
  Tensor hdr_rec;
  if (ne && hdr_on) hdr_rec = torch::empty({std::max<int64_t>(1, hdr_pos) * 16}, dev_opts.dtype(torch::kUInt8));
  if (ne) dec = torch::empty({dec_pos + kAlign}, dev_opts.dtype(torch::kUInt8));
  clk.lap(kStAlloc);
  if (ne) {
    hip_ok(hlsp2p::dev::launch_aes128_cbc_decrypt(
               static_cast<const uint8_t*>(src.data_ptr()), static_cast<uint8_t*>(dec.data_ptr()),
               desc.at<int64_t>(d_so), desc.at<int64_t>(d_do), desc.at<int64_t>(d_bp), desc.at<int64_t>(d_cp),
               desc.at<uint32_t>(d_drk), desc.at<uint32_t>(d_iv), static_cast<const uint32_t*>(td0.data_ptr()),
               static_cast<const uint8_t*>(isb.data_ptr()), out_len.data_ptr<int64_t>(), static_cast<int>(ne),
               a_cp.back(), decrypt_cus(device), st, nv ? desc.at<int64_t>(d_mo) : nullptr,
               nv ? crc_w->data_ptr() : nullptr, nv ? reinterpret_cast<uint32_t*>(masks.data_ptr<int32_t>()) : nullptr,
               hdr_on ? desc.at<int64_t>(d_ho) : nullptr, hdr_on ? hdr_rec.data_ptr() : nullptr),
           "aes128_cbc_decrypt");
  }
  if (nv) {  // fold the decrypt's CRC masks per chunk, combine per segment, compare
    hip_ok(hlsp2p::dev::launch_crc32_from_masks(
               reinterpret_cast<const uint32_t*>(masks.data_ptr<int32_t>()),
               static_cast<const uint8_t*>(crc_w->data_ptr()) + 8 * 64 * 16, desc.at<int64_t>(d_vco),
               desc.at<int64_t>(d_vl), static_cast<const uint32_t*>(crc_tables->data_ptr()),
               reinterpret_cast<uint32_t*>(chunk_res.data_ptr<int32_t>()),
               reinterpret_cast<uint32_t*>(v_crc.data_ptr<int32_t>()), desc.at<uint32_t>(d_vx),
               v_ok.data_ptr<uint8_t>(), nullptr, nullptr, 0, static_cast<int>(nv), v_chunks, cus(device), st),
           "crc32_from_masks");
    v_ok_host = torch::empty({nv}, torch::TensorOptions().dtype(torch::kUInt8).pinned_memory(true));
    v_ok_host.copy_(v_ok, /*non_blocking=*/true);
  }
  clk.lap(kStDecrypt);

  py::list groups, keep;  // keep: scratch the kernels use until the batch completes
  int64_t row0 = 0;
  for (int g = 0; g < 2; ++g) {
    DemuxPlan& p = g == 0 ? pe : pc;
    const int64_t n = static_cast<int64_t>(p.idx.size());
    if (!n) continue;
    const uint8_t* buf = g == 1 ? static_cast<const uint8_t*>(src.data_ptr())
                         : dec.defined() ? static_cast<const uint8_t*>(dec.data_ptr()) : nullptr;
    const int64_t* lens = g == 0 ? out_len.data_ptr<int64_t>() : desc.at<int64_t>(p.d_len);
    const int64_t nb_blocks = std::max<int64_t>(1, p.total_blocks);
    Tensor es = torch::empty({p.es_bytes}, dev_opts.dtype(torch::kUInt8));
    Tensor info = torch::empty({n, kInfo}, dev_opts.dtype(torch::kInt64));
    Tensor pes = torch::empty({n, 3, max_pes, 3}, dev_opts.dtype(torch::kInt64));
    Tensor meta = torch::empty({nb_blocks * 256}, dev_opts.dtype(torch::kInt32));
    Tensor pts = torch::empty({nb_blocks * 256 * 2}, dev_opts.dtype(torch::kInt64));
    Tensor aux = torch::empty({nb_blocks * 12 + n * 7}, dev_opts.dtype(torch::kInt32));
    hip_ok(hlsp2p::dev::launch_ts_demux(buf, desc.at<int64_t>(p.d_off), lens, desc.at<int64_t>(p.d_bp),
                                        static_cast<int>(n), p.total_blocks,
                                        reinterpret_cast<uint32_t*>(meta.data_ptr<int32_t>()),
                                        pts.data_ptr<int64_t>(), aux.data_ptr<int32_t>(), es.data_ptr<uint8_t>(),
                                        desc.at<int64_t>(p.d_eo), pes.data_ptr<int64_t>(), max_pes,
                                        info.data_ptr<int64_t>(), st,
                                        g == 0 && hdr_on ? hdr_rec.data_ptr() : nullptr,
                                        g == 0 && hdr_on ? desc.at<int64_t>(d_ho) : nullptr),
           "ts_demux");
    keep.append(py::make_tuple(meta, pts, aux));
    // D2H through torch's copy so the caching host allocator records the use of the pinned
    // block on `st` (it is not handed out again before the copy has run, even if the batch
    // is dropped uncompleted)
    Tensor hinfo = host.narrow(0, row0 * kInfo, n * kInfo).view({n, kInfo});
    hinfo.copy_(info, /*non_blocking=*/true);
    py::object hlens;
    if (g == 0) {
      Tensor hl = host.narrow(0, (ne + nc) * kInfo, ne);
      hl.copy_(out_len, /*non_blocking=*/true);
      hlens = py::cast(hl);
    } else {
      I64 l(static_cast<py::ssize_t>(n));
      std::memcpy(l.mutable_data(), p.len.data(), static_cast<size_t>(n * 8));
      hlens = l;
    }
    I64 idx(static_cast<py::ssize_t>(n)), eo(static_cast<py::ssize_t>(n));
    std::memcpy(idx.mutable_data(), p.idx.data(), static_cast<size_t>(n * 8));
    std::memcpy(eo.mutable_data(), p.es_off.data(), static_cast<size_t>(n * 8));
    groups.append(py::make_tuple(idx, info, pes, es, eo, hinfo, hlens));
    row0 += n;
  }
  clk.lap(kStDemux);
  keep.append(dec.defined() ? py::cast(dec) : py::none());
  keep.append(desc.device());
  if (hdr_rec.defined()) keep.append(hdr_rec);
  py::object verify = py::none();
  if (nv) {
    keep.append(py::make_tuple(masks, chunk_res, v_crc, v_ok));
    I64 vi(static_cast<py::ssize_t>(nv));
    std::memcpy(vi.mutable_data(), v_idx.data(), static_cast<size_t>(nv * 8));
    verify = py::make_tuple(vi, v_ok_host);  // batch indices of the verified segments, ok flags (pinned)
  }
  auto out = py::make_tuple(groups, keep, host, verify);
  clk.lap(kStResult);
  return out;
}

}  // namespace

void register_transmux(py::module& m) {
  m.def("set_cu_reserve", [](int n) { g_cu_reserve = std::max(0, n); }, py::arg("n"),
        "CUs the persistent decrypt grid leaves free for concurrent (RCCL) kernels");
  m.def("cu_reserve", [] { return g_cu_reserve; });
  m.def(
      "transmux_launch_profile",
      [](bool reset) {
        py::dict d;
        const char* names[kStages] = {"plan",          "desc_build",       "alloc",      "decrypt_launch",
                                      "demux_launch_d2h", "results",       "desc_pinned", "desc_memcpy",
                                      "desc_dev_alloc",   "desc_h2d"};
        for (int i = 0; i < kStages; ++i) d[names[i]] = g_stage_us[i];
        d["calls"] = g_calls;
        if (reset) {
          g_stage_us.fill(0.0);
          g_calls = 0;
        }
        return d;
      },
      py::arg("reset") = false, "host microseconds of transmux_launch by stage (summed) and the call count");
  m.def("transmux_launch", &transmux_launch, py::arg("src"), py::arg("src_off"), py::arg("nbytes"), py::arg("enc"),
        py::arg("drk"), py::arg("iv"), py::arg("td0"), py::arg("isb"), py::arg("max_pes"),
        py::arg("expect") = py::none(), py::arg("crc_w") = py::none(), py::arg("crc_tables") = py::none());
}
