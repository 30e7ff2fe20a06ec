// Node-local shared-memory sample store (host side, POSIX shm) — the single-node
// replacement of pyddstore's one-sided MPI RMA store (reference
// hydragnn/utils/datasets/distdataset.py:22-183).
//
// Every rank serialises its shard of samples into one shm segment
// (/dev/shm/<name>); any rank on the node maps any segment read-only and copies a
// sample's byte range out (or gets a zero-copy view).  On one MI355X node all 8
// ranks share host memory, so "remote gets" are plain memcpy from the page cache —
// no RMA windows, no epoch fences.  Handles index a process-local table.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include <ATen/ATen.h>
#include <torch/library.h>

namespace hy {
namespace {

struct Seg {
  std::string name;
  void* base = nullptr;
  int64_t size = 0;
  bool writable = false;
};

std::mutex g_mu;
std::vector<Seg> g_segs;

std::string shm_name(const std::string& n) { return n.empty() || n[0] == '/' ? n : "/" + n; }

int64_t add_seg(Seg s) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (size_t i = 0; i < g_segs.size(); ++i)
    if (g_segs[i].base == nullptr) {
      g_segs[i] = s;
      return (int64_t)i;
    }
  g_segs.push_back(s);
  return (int64_t)g_segs.size() - 1;
}

Seg& get_seg(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(h >= 0 && h < (int64_t)g_segs.size() && g_segs[h].base != nullptr, "shm_store: bad handle ", h);
  return g_segs[h];
}

}  // namespace

int64_t shm_store_create(const std::string& name, int64_t nbytes) {
  TORCH_CHECK(nbytes >= 0, "shm_store_create: negative size");
  const std::string n = shm_name(name);
  int fd = shm_open(n.c_str(), O_CREAT | O_RDWR | O_TRUNC, 0600);
  TORCH_CHECK(fd >= 0, "shm_open(", n, ") failed: ", std::strerror(errno));
  const int64_t sz = std::max<int64_t>(nbytes, 1);
  if (ftruncate(fd, sz) != 0) {
    close(fd);
    shm_unlink(n.c_str());
    TORCH_CHECK(false, "ftruncate(", n, ", ", sz, ") failed: ", std::strerror(errno));
  }
  void* p = mmap(nullptr, sz, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  TORCH_CHECK(p != MAP_FAILED, "mmap(", n, ") failed: ", std::strerror(errno));
  return add_seg(Seg{n, p, nbytes, true});
}

int64_t shm_store_attach(const std::string& name) {
  const std::string n = shm_name(name);
  int fd = shm_open(n.c_str(), O_RDONLY, 0);
  TORCH_CHECK(fd >= 0, "shm_open(", n, ") for attach failed: ", std::strerror(errno));
  struct stat st;
  fstat(fd, &st);
  const int64_t sz = std::max<int64_t>(st.st_size, 1);
  void* p = mmap(nullptr, sz, PROT_READ, MAP_SHARED, fd, 0);
  close(fd);
  TORCH_CHECK(p != MAP_FAILED, "mmap(", n, ") failed: ", std::strerror(errno));
  return add_seg(Seg{n, p, (int64_t)st.st_size, false});
}

void shm_store_write(int64_t h, int64_t offset, const at::Tensor& src) {
  Seg& s = get_seg(h);
  TORCH_CHECK(s.writable, "shm_store_write: segment attached read-only");
  TORCH_CHECK(src.device().is_cpu() && src.is_contiguous(), "shm_store_write: contiguous CPU tensor expected");
  const int64_t nb = src.numel() * (int64_t)src.element_size();
  TORCH_CHECK(offset >= 0 && offset + nb <= s.size, "shm_store_write: range [", offset, ", ", offset + nb,
              ") outside segment of ", s.size, " bytes");
  std::memcpy(static_cast<char*>(s.base) + offset, src.data_ptr(), nb);
}

at::Tensor shm_store_read(int64_t h, int64_t offset, int64_t nbytes) {
  Seg& s = get_seg(h);
  TORCH_CHECK(offset >= 0 && nbytes >= 0 && offset + nbytes <= s.size, "shm_store_read: range [", offset, ", ",
              offset + nbytes, ") outside segment of ", s.size, " bytes");
  auto out = at::empty({nbytes}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(out.data_ptr(), static_cast<const char*>(s.base) + offset, nbytes);
  return out;
}

// Zero-copy uint8 view; valid until shm_store_close(h).
at::Tensor shm_store_view(int64_t h, int64_t offset, int64_t nbytes) {
  Seg& s = get_seg(h);
  TORCH_CHECK(offset >= 0 && nbytes >= 0 && offset + nbytes <= s.size, "shm_store_view: range outside segment");
  return at::from_blob(static_cast<char*>(s.base) + offset, {nbytes}, at::TensorOptions().dtype(at::kByte));
}

int64_t shm_store_size(int64_t h) { return get_seg(h).size; }

void shm_store_close(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(h >= 0 && h < (int64_t)g_segs.size(), "shm_store_close: bad handle");
  Seg& s = g_segs[h];
  if (s.base) munmap(s.base, std::max<int64_t>(s.size, 1));
  s = Seg{};
}

void shm_store_unlink(const std::string& name) { shm_unlink(shm_name(name).c_str()); }

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("shm_store_create(str name, int nbytes) -> int", hy::shm_store_create);
  m.def("shm_store_attach(str name) -> int", hy::shm_store_attach);
  m.def("shm_store_write(int h, int offset, Tensor src) -> ()", hy::shm_store_write);
  m.def("shm_store_read(int h, int offset, int nbytes) -> Tensor", hy::shm_store_read);
  m.def("shm_store_view(int h, int offset, int nbytes) -> Tensor", hy::shm_store_view);
  m.def("shm_store_size(int h) -> int", hy::shm_store_size);
  m.def("shm_store_close(int h) -> ()", hy::shm_store_close);
  m.def("shm_store_unlink(str name) -> ()", hy::shm_store_unlink);
}
