// Check of an exact-division shortcut measured and dropped in round 4 (profiles/r04/ab_div_runs_dropped.txt):
// div_by restated for the host, against a / d: random bit patterns over the whole
// float range (edge cases take the plain division) and scene-like operands
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdint>
#include <random>
#include <thread>
#include <vector>
#include <atomic>
static float F(uint32_t u){float f;memcpy(&f,&u,4);return f;}
static uint32_t U(float f){uint32_t u;memcpy(&u,&f,4);return u;}
static float div_by(float a, float d, float y) {
  const float ad = std::fabs(d), aa = std::fabs(a);
  if (ad >= 0x1p-60f && ad <= 0x1p60f && (a == 0.0f || (aa >= 0x1p-60f && aa <= 0x1p60f))) {
    const float q = a * y;
    return a == 0.0f ? q : std::fma(std::fma(-d, q, a), y, q);
  }
  return a / d;
}
int main(){
  std::atomic<long long> bad{0}, tot{0};
  std::vector<std::thread> th;
  for(int t=0;t<16;++t) th.emplace_back([&,t]{
    std::mt19937 rng(777+t);
    long long b=0,n=0;
    for(long long i=0;i<200000000LL;++i){
      float a, d;
      uint32_t ra=rng(), rd=rng();
      switch (i % 3) {
        case 0: a = F(ra); d = F(rd); break;                                   // any bit pattern
        case 1: a = F((ra & 0x807fffffu) | ((60u + (ra>>24)%136u) << 23));     // around the guard edges
                d = F((rd & 0x807fffffu) | ((60u + (rd>>24)%136u) << 23)); break;
        default: a = std::ldexp((float)(ra>>8), -24) * 2e4f - 1e4f;            // scene-like
                 d = std::ldexp((float)(rd>>8), -24) * 2.f - 1.f; if (ra & 1) a = 0.f * a; break;
      }
      const float y = 1.0f / d;
      const float got = div_by(a, d, y), want = a / d;
      ++n;
      if (U(got) != U(want) && !(got != got && want != want)) { if (b < 5) printf("a=%a d=%a got %a want %a\n", a, d, got, want); ++b; }
    }
    bad += b; tot += n;
  });
  for(auto&x:th) x.join();
  printf("div_by vs a / d: %lld of %lld differ (random bit patterns, guard edges, scene-like operands incl. signed zeros)\n", bad.load(), tot.load());
}
