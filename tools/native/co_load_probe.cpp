// Where does loading a large code object go?  hipModuleLoadData on a gfx950
// code object file, then hipModuleGetFunction + one attribute query for every
// kernel it defines (the *.kd symbols), each phase timed.  Used on RCCL's
// 569 MB gfx950 code object (tools/rccl_init_probe.py: the "kernels" phase).
#include <elf.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <unistd.h>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                               \
    }                                                                         \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  double t0 = now();
  std::ifstream f(argv[1], std::ios::binary);
  std::vector<char> co((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  double t_read = now() - t0;
  // kernel names from the ELF symbol tables
  std::vector<std::string> kernels;
  auto* eh = reinterpret_cast<const Elf64_Ehdr*>(co.data());
  if (co.size() < sizeof(Elf64_Ehdr) || memcmp(eh->e_ident, ELFMAG, SELFMAG) != 0) return 3;
  auto* sh = reinterpret_cast<const Elf64_Shdr*>(co.data() + eh->e_shoff);
  for (int i = 0; i < eh->e_shnum; ++i) {
    if (sh[i].sh_type != SHT_SYMTAB && sh[i].sh_type != SHT_DYNSYM) continue;
    const char* str = co.data() + sh[sh[i].sh_link].sh_offset;
    auto* sym = reinterpret_cast<const Elf64_Sym*>(co.data() + sh[i].sh_offset);
    for (size_t j = 0; j < sh[i].sh_size / sizeof(Elf64_Sym); ++j) {
      std::string n = str + sym[j].st_name;
      if (n.size() > 3 && n.compare(n.size() - 3, 3, ".kd") == 0) kernels.push_back(n.substr(0, n.size() - 3));
    }
    if (sh[i].sh_type == SHT_DYNSYM) break;
  }
  double t1 = now();
  CHECK(hipSetDevice(0));
  CHECK(hipFree(nullptr));
  double t_init = now() - t1;
  t1 = now();
  hipModule_t m;
  CHECK(hipModuleLoadData(&m, co.data()));
  double t_load = now() - t1;
  t1 = now();
  std::vector<hipFunction_t> fns;
  for (auto& k : kernels) {
    hipFunction_t fn;
    if (hipModuleGetFunction(&fn, m, k.c_str()) == hipSuccess) fns.push_back(fn);
  }
  double t_get = now() - t1;
  t1 = now();
  long long regs = 0;
  for (auto fn : fns) {
    int v = 0;
    if (hipFuncGetAttribute(&v, HIP_FUNC_ATTRIBUTE_NUM_REGS, fn) == hipSuccess) regs += v;
  }
  double t_attr = now() - t1;
  printf("{\"bytes\": %zu, \"kernels\": %zu, \"found\": %zu, \"read_s\": %.4f, \"hip_init_s\": %.4f, "
         "\"module_load_s\": %.4f, \"get_function_s\": %.4f, \"attributes_s\": %.4f, \"regs_sum\": %lld}\n",
         co.size(), kernels.size(), fns.size(), t_read, t_init, t_load, t_get, t_attr, regs);
  fflush(stdout);
  _exit(0);
}
