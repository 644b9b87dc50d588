#include <chrono>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cmath>
namespace cusz_amd { int build_codebook(const uint32_t* hist, int bklen, uint32_t* book, uint8_t* revbook); }
int main(){
  std::vector<uint32_t> h(1024);
  for(int s=0;s<1024;s++){ double d=(s-512)/6.0; double v=1.3e8*std::exp(-d*d/2)/15.0; if (std::abs(s-512)<330) v+= 20; h[s]=(uint32_t)v; }
  std::vector<uint32_t> book(1024); std::vector<uint8_t> rv(4096);
  for(int w=0;w<50;w++) cusz_amd::build_codebook(h.data(),1024,book.data(),rv.data());
  auto t0=std::chrono::steady_clock::now();
  for(int w=0;w<1000;w++) cusz_amd::build_codebook(h.data(),1024,book.data(),rv.data());
  auto t1=std::chrono::steady_clock::now();
  printf("%.2f us per book\n", std::chrono::duration<double,std::micro>(t1-t0).count()/1000);
}
