// ASan driver for the fast-path bodies: fast_host_asan PROGRAM.json N KEYS BATCH
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>
extern "C" {
void* fh_create(const char*, int, long, long);
int fh_push(void*, long, const long*, const int*, const int*, const void* const*, const unsigned char* const*);
long fh_num_matches(void*);
}
int main(int argc, char** argv) {
  std::ifstream f(argv[1]);
  std::stringstream ss; ss << f.rdbuf();
  long n = atol(argv[2]); int keys = atoi(argv[3]); long batch = atol(argv[4]);
  void* h = fh_create(ss.str().c_str(), keys, batch, 1 << 20);
  if (!h) { printf("create failed\n"); return 1; }
  unsigned long long s = 12345;
  std::vector<long> ts(n); std::vector<int> key(n), st(n, 0); std::vector<float> price(n);
  for (long i = 0; i < n; i++) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    key[i] = (int)((s >> 33) % keys); price[i] = (float)((s >> 20) % 10000) / 100.0f;
    ts[i] = 1544512385000L + (keys > 100 ? i / (keys / 100) : i);
  }
  for (long lo = 0; lo < n; lo += batch) {
    long m = std::min(batch, n - lo);
    const void* cols[1] = {price.data() + lo};
    int rc = fh_push(h, m, ts.data() + lo, key.data() + lo, st.data() + lo, cols, nullptr);
    if (rc) { printf("push rc %d\n", rc); return 2; }
  }
  printf("ok matches %ld\n", fh_num_matches(h));
  return 0;
}
