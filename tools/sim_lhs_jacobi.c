// Jacobi decode of the numpy shuffle rejection stream: convergence passes (simulation only)
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <math.h>
#include <string.h>
static uint64_t sm(uint64_t *x){uint64_t z=(*x+=0x9E3779B97F4A7C15ull);z=(z^(z>>30))*0xBF58476D1CE4E5B9ull;z=(z^(z>>27))*0x94D049BB133111EBull;return z^(z>>31);}
static int64_t N1, D; static int64_t n;
static inline uint32_t maskof(uint32_t i){uint32_t m=i;m|=m>>1;m|=m>>2;m|=m>>4;m|=m>>8;m|=m>>16;return m;}
// state g in [0, D*N1]; returns new state after L draws
static int64_t walk(const uint32_t* w, int64_t L, int64_t g){
  int64_t total=D*N1;
  for(int64_t t=0;t<L && g<total;t++){
    int64_t i = n-1-(g%N1);
    uint32_t m=maskof((uint32_t)i);
    if((w[t]&m) <= (uint32_t)i) g++;
  }
  return g;
}
int main(int argc,char**argv){
  n=atoll(argv[1]); D=atoll(argv[2]); int64_t L=atoll(argv[3]);
  N1=n-1;
  // expected draws per column
  double Ecol=0; for(int64_t i=1;i<n;i++) Ecol += (double)(maskof(i)+1)/(i+1);
  int64_t T=(int64_t)(Ecol*D + 64*sqrt(Ecol*D)+4096);
  uint32_t* w=malloc(T*4); uint64_t x=12345; for(int64_t t=0;t<T;t++) w[t]=(uint32_t)sm(&x);
  // exact sequential
  int64_t K=(T+L-1)/L; int64_t* ex=malloc((K+1)*8); int64_t g=0;
  for(int64_t k=0;k<K;k++){ex[k]=g; g=walk(w+k*L, (k==K-1)?T-k*L:L, g);} ex[K]=g;
  printf("T=%lld K=%lld final=%lld need=%lld\n",(long long)T,(long long)K,(long long)g,(long long)(D*N1));
  // initial guess: expected state at draw t: per-column cumulative expected draws, inverted numerically via table
  double* cum=malloc(n*sizeof(double)); // cum[s] = expected draws to reach step s (s steps done) within column
  cum[0]=0; for(int64_t s=0;s<N1;s++){int64_t i=n-1-s; cum[s+1]=cum[s]+(double)(maskof(i)+1)/(i+1);} 
  int64_t* st=malloc(K*8); int64_t* cnt=malloc(K*8);
  for(int64_t k=0;k<K;k++){double t=(double)k*L; int64_t c=(int64_t)(t/Ecol); double r=t-c*Ecol; if(c>=D){st[k]=D*N1;continue;}
    int64_t lo=0,hi=N1; while(lo<hi){int64_t mid=(lo+hi+1)/2; if(cum[mid]<=r) lo=mid; else hi=mid-1;} st[k]=c*N1+lo; }
  st[0]=0;
  for(int pass=1;pass<=400;pass++){
    int64_t maxerr=0, nerr=0; for(int64_t k=0;k<K;k++){int64_t e=llabs(st[k]-ex[k]); if(e){nerr++; if(e>maxerr)maxerr=e;}}
    if(pass<=12 || pass%10==0 || nerr==0) printf("pass %d: wrong starts %lld max err %lld\n",pass,(long long)nerr,(long long)maxerr);
    if(nerr==0) break;
    for(int64_t k=0;k<K;k++) cnt[k]=walk(w+k*L,(k==K-1)?T-k*L:L,st[k])-st[k];
    int64_t acc=0; for(int64_t k=0;k<K;k++){st[k]=acc; acc+=cnt[k];}
  }
  return 0;
}
