// Swarm-node host path, native (agent/node.py, SURVEY §2.2 K3 + K12):
//
// * crc32_launch — the MFMA CRC-32 of a round's segments in one call: descriptor math,
//   one staging H2D, residue + combine launches (kernels/crc32_mfma.hip), optional verify
//   against expected values and scatter into the per-entry CRC table.  The Python path
//   (numpy prefix sums, a descriptor pack, three allocations, a pybind launch) cost ~45 us
//   per call; a round calls it once (CDN ingest) or twice (+ P2P verify).
// * arena_views — the zero-copy uint8 views of the HBM arena handed to the loaders, made
//   in one call (a Python slice costs ~1.5 us each, 64+ per round).
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>
#include <torch/extension.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include <cstring>
#include <vector>

namespace hlsp2p {
namespace dev {
hipError_t launch_crc32_batch(const uint8_t*, const int64_t*, const int64_t*, const int64_t*, const int64_t*,
                              const void*, const uint32_t*, uint32_t*, uint32_t*, const uint32_t*, uint8_t*,
                              const int64_t*, uint32_t*, int64_t, int, int64_t, int, bool, hipStream_t,
                              const int64_t*);
}  // namespace dev
}  // namespace hlsp2p

namespace {

namespace py = pybind11;
using torch::Tensor;
using I64 = py::array_t<int64_t, py::array::c_style | py::array::forcecast>;

int cus(int device) {
  static int cached[64] = {0};
  if (device >= 0 && device < 64 && cached[device]) return cached[device];
  int n = 0;
  hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device);
  if (n <= 0) n = 256;
  if (device >= 0 && device < 64) cached[device] = n;
  return n;
}

void put(std::vector<uint8_t>& blk, int64_t& off, const void* p, int64_t nbytes) {
  off = static_cast<int64_t>(blk.size());
  blk.resize(off + ((nbytes + 15) & ~int64_t(15)), 0);
  if (nbytes) std::memcpy(blk.data() + off, p, static_cast<size_t>(nbytes));
}

// CRC-32 (zlib) of buf[offs[i] : offs[i] + lens[i]] (16-byte aligned offsets).  `expect`:
// int32 device tensor of expected values -> also returns ok (uint8, 1 = match).  `scatter_to`
// / `scatter_idx`: the combine kernel writes crc[i] to scatter_to[scatter_idx[i]] (ids ride
// the descriptor block).  `wfrag` selects the matrix-core path (see crc32_batch).  `keys`
// (int64[B, 4] segment keys, riding the descriptor block): keyed mode -- `expect` and the
// scattered table values are the CRCs bound to each segment's key (crc ^ key_digest); the
// returned crc stays the plain CRC-32.
py::tuple crc32_launch(Tensor buf, I64 offs, I64 lens, Tensor wfrag, Tensor tables, c10::optional<Tensor> expect,
                       c10::optional<Tensor> scatter_to, c10::optional<I64> scatter_idx, c10::optional<I64> keys) {
  TORCH_CHECK_VALUE(buf.is_cuda() && buf.is_contiguous() && buf.scalar_type() == torch::kUInt8, "buf: contiguous GPU uint8");
  TORCH_CHECK_VALUE((reinterpret_cast<uintptr_t>(buf.data_ptr()) & 15) == 0, "buf must be 16-byte aligned");
  const int64_t B = offs.size();
  TORCH_CHECK_VALUE(lens.size() == B, "crc32_launch: offs / lens sizes differ");
  const bool fp4 = wfrag.scalar_type() == torch::kUInt8;
  TORCH_CHECK_VALUE(wfrag.is_cuda() && wfrag.numel() >= (fp4 ? 32 * 64 * 16 : 64 * 64 * 16), "wfrag");
  TORCH_CHECK_VALUE(tables.is_cuda() && tables.scalar_type() == torch::kInt32 && tables.numel() >= 48 * 1024, "tables");
  const int device = buf.get_device();
  const auto dev_opts = torch::TensorOptions().device(torch::kCUDA, device);
  if (B == 0)
    return py::make_tuple(torch::empty({0}, dev_opts.dtype(torch::kInt32)),
                          expect.has_value() ? py::cast(torch::empty({0}, dev_opts.dtype(torch::kUInt8))) : py::none());
  const int64_t* o = offs.data();
  const int64_t* n = lens.data();
  const int64_t cap = buf.numel();
  std::vector<int64_t> tile_prefix(B + 1, 0), res_off(B, 0);
  int64_t groups_total = 0;
  for (int64_t i = 0; i < B; ++i) {
    TORCH_CHECK_VALUE(o[i] >= 0 && n[i] >= 0 && o[i] + n[i] <= cap, "crc32_launch: range out of bounds");
    TORCH_CHECK_VALUE(o[i] % 16 == 0, "crc32_launch: offsets must be 16-byte aligned");
    const int64_t groups = (n[i] + 255) / 256;
    res_off[i] = groups_total;
    groups_total += groups;
    tile_prefix[i + 1] = tile_prefix[i] + (groups + 31) / 32;
  }
  const uint32_t* ex = nullptr;
  if (expect.has_value()) {
    TORCH_CHECK_VALUE(expect->is_cuda() && expect->scalar_type() == torch::kInt32 && expect->numel() >= B &&
                    expect->is_contiguous(),
                "expect: int32 GPU tensor of B values");
    ex = static_cast<const uint32_t*>(expect->data_ptr());
  }
  TORCH_CHECK_VALUE(scatter_to.has_value() == scatter_idx.has_value(), "scatter_to and scatter_idx go together");
  std::vector<uint8_t> blk;
  int64_t d_o, d_n, d_tp, d_ro, d_si = -1, d_k = -1;
  put(blk, d_o, o, B * 8);
  put(blk, d_n, n, B * 8);
  put(blk, d_tp, tile_prefix.data(), (B + 1) * 8);
  put(blk, d_ro, res_off.data(), B * 8);
  uint32_t* sout = nullptr;
  int64_t sn = 0;
  if (scatter_to.has_value()) {
    TORCH_CHECK_VALUE(scatter_to->is_cuda() && scatter_to->scalar_type() == torch::kInt32 && scatter_to->is_contiguous(),
                "scatter_to: int32 GPU tensor");
    const I64& si = *scatter_idx;
    TORCH_CHECK_VALUE(si.size() == B, "scatter_idx size");
    sn = scatter_to->numel();
    for (int64_t i = 0; i < B; ++i) TORCH_CHECK_VALUE(si.data()[i] >= 0 && si.data()[i] < sn, "scatter index out of range");
    put(blk, d_si, si.data(), B * 8);
    sout = static_cast<uint32_t*>(scatter_to->data_ptr());
  }
  if (keys.has_value()) {
    TORCH_CHECK_VALUE(keys->size() == 4 * B, "keys: int64[B, 4]");
    put(blk, d_k, keys->data(), B * 32);
  }
  const int64_t nbytes = static_cast<int64_t>(blk.size());
  Tensor host = torch::empty({nbytes}, torch::TensorOptions().dtype(torch::kUInt8).pinned_memory(true));
  std::memcpy(host.data_ptr<uint8_t>(), blk.data(), blk.size());
  // one device block: descriptors | residues | crc | ok
  const int64_t res_words = std::max<int64_t>(1, groups_total);
  const int64_t d_res = (nbytes + 255) / 256 * 256;
  const int64_t d_crc = d_res + (res_words * 4 + 255) / 256 * 256;
  const int64_t d_ok = d_crc + (B * 4 + 255) / 256 * 256;
  Tensor dblk = torch::empty({d_ok + B}, dev_opts.dtype(torch::kUInt8));
  dblk.narrow(0, 0, nbytes).copy_(host, /*non_blocking=*/true);
  uint8_t* base = dblk.data_ptr<uint8_t>();
  auto at = [&](int64_t off) { return reinterpret_cast<int64_t*>(base + off); };
  Tensor crc = dblk.narrow(0, d_crc, B * 4).view(torch::kInt32);
  Tensor ok = dblk.narrow(0, d_ok, B);
  hipStream_t st = c10::hip::getCurrentHIPStream(device).stream();
  const hipError_t e = hlsp2p::dev::launch_crc32_batch(
      static_cast<const uint8_t*>(buf.data_ptr()), at(d_o), at(d_n), at(d_tp), at(d_ro), wfrag.data_ptr(),
      static_cast<const uint32_t*>(tables.data_ptr()), reinterpret_cast<uint32_t*>(base + d_res),
      reinterpret_cast<uint32_t*>(base + d_crc), ex, ex ? base + d_ok : nullptr, d_si >= 0 ? at(d_si) : nullptr, sout,
      sn, static_cast<int>(B), tile_prefix[B], cus(device), fp4, st, d_k >= 0 ? at(d_k) : nullptr);
  TORCH_CHECK(e == hipSuccess, "crc32 launch failed: ", hipGetErrorString(e));
  return py::make_tuple(crc, ex ? py::cast(ok) : py::none());
}

// 1-D uint8 views arena[offs[i] : offs[i] + lens[i]] (shared storage, no copy).
std::vector<Tensor> arena_views(const Tensor& arena, I64 offs, I64 lens) {
  TORCH_CHECK_VALUE(arena.dim() == 1 && arena.is_contiguous(), "arena must be a contiguous 1-D tensor");
  const int64_t B = offs.size();
  TORCH_CHECK_VALUE(lens.size() == B, "arena_views: offs / lens sizes differ");
  const int64_t* o = offs.data();
  const int64_t* n = lens.data();
  const int64_t cap = arena.numel();
  std::vector<Tensor> out;
  out.reserve(static_cast<size_t>(B));
  for (int64_t i = 0; i < B; ++i) {
    TORCH_CHECK_VALUE(o[i] >= 0 && n[i] >= 0 && o[i] + n[i] <= cap, "arena_views: range out of bounds");
    out.push_back(arena.narrow(0, o[i], n[i]));
  }
  return out;
}

}  // namespace

void register_ingest(py::module& m) {
  m.def("crc32_launch", &crc32_launch, py::arg("buf"), py::arg("offs"), py::arg("lens"), py::arg("wfrag"),
        py::arg("tables"), py::arg("expect") = py::none(), py::arg("scatter_to") = py::none(),
        py::arg("scatter_idx") = py::none(), py::arg("keys") = py::none());
  m.def("arena_views", &arena_views, py::arg("arena"), py::arg("offs"), py::arg("lens"));
}
