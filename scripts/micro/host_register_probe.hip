// Probe: can a file's page-cache pages be DMA'd to the GPU directly
// (mmap + hipHostRegister), and what do registration and the copy cost
// against fread into pinned memory?  ./host_register_probe [MB] [files]
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>
#include <chrono>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); } } while (0)

int main(int argc, char **argv) {
  const size_t mb = argc > 1 ? atoi(argv[1]) : 25, nf = argc > 2 ? atoi(argv[2]) : 8;
  const size_t n = mb << 20;
  const char *dir = getenv("TMPDIR") ? getenv("TMPDIR") : "/tmp";
  std::vector<std::string> paths;
  std::vector<char> buf(n, 7);
  for (size_t i = 0; i < nf; i++) {
    char p[512];
    snprintf(p, sizeof p, "%s/hrp_%zu.bin", dir, i);
    FILE *f = fopen(p, "wb");
    fwrite(buf.data(), 1, n, f);
    fclose(f);
    paths.push_back(p);
  }
  uint8_t *d = nullptr, *pin = nullptr;
  CK(hipMalloc(&d, n));
  CK(hipHostMalloc((void **)&pin, n, hipHostMallocDefault));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  for (int rep = 0; rep < 3; rep++) {
    double t_reg = 0, t_cp = 0, t_unreg = 0, t_rd = 0, t_cp2 = 0;
    int ok = 1;
    for (size_t i = 0; i < nf; i++) {
      int fd = open(paths[i].c_str(), O_RDONLY);
      double t0 = now();
      void *m = mmap(nullptr, n, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, 0);
      hipError_t e = hipHostRegister(m, n, hipHostRegisterReadOnly);
      double t1 = now();
      if (e != hipSuccess) {
        if (rep == 0 && i == 0) printf("hipHostRegister(file mmap): %s\n", hipGetErrorString(e));
        ok = 0;
      } else {
        void *dp = nullptr;
        CK(hipHostGetDevicePointer(&dp, m, 0));
        CK(hipMemcpyAsync(d, m, n, hipMemcpyHostToDevice, st));
        CK(hipStreamSynchronize(st));
      }
      double t2 = now();
      if (e == hipSuccess) CK(hipHostUnregister(m));
      munmap(m, n);
      close(fd);
      double t3 = now();
      t_reg += t1 - t0; t_cp += t2 - t1; t_unreg += t3 - t2;
      // the fread path
      double t4 = now();
      FILE *f = fopen(paths[i].c_str(), "rb");
      if (fread(pin, 1, n, f) != n) printf("short read\n");
      fclose(f);
      double t5 = now();
      CK(hipMemcpyAsync(d, pin, n, hipMemcpyHostToDevice, st));
      CK(hipStreamSynchronize(st));
      double t6 = now();
      t_rd += t5 - t4; t_cp2 += t6 - t5;
    }
    printf("rep %d, %zu files of %zu MB: mmap+register %.2f ms/file, copy %.2f ms/file (%.1f GB/s), unregister+munmap %.2f ms/file%s; "
           "fread into pinned %.2f ms/file (%.1f GB/s), copy %.2f ms/file (%.1f GB/s)\n",
           rep, nf, mb, 1e3 * t_reg / nf, 1e3 * t_cp / nf, ok ? n * nf / t_cp / 1e9 : 0.0, 1e3 * t_unreg / nf,
           ok ? "" : " (register FAILED)", 1e3 * t_rd / nf, n * nf / t_rd / 1e9, 1e3 * t_cp2 / nf, n * nf / t_cp2 / 1e9);
  }
  for (auto &p : paths) unlink(p.c_str());
  return 0;
}
