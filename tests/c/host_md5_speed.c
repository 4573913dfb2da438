/* Host per-message MD5 speed (MD5Init/Update/Final per message, md5.h:41-51):
 * linked against libmd5hip's md5_stream.c or against the reference md5.c
 * compiled in place, by scripts/host_md5_speed.sh.  Bench tool, not a test. */
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <time.h>
struct MD5Context { uint32_t buf[4]; uint32_t bits[2]; unsigned char in[64]; };
void MD5Init(struct MD5Context *); void MD5Update(struct MD5Context *, const void *, unsigned); void MD5Final(unsigned char *, struct MD5Context *);
static double now(){struct timespec t; clock_gettime(CLOCK_MONOTONIC,&t); return t.tv_sec+t.tv_nsec*1e-9;}
int main(int argc, char**argv){
  size_t L = argc>1? strtoul(argv[1],0,0):16384; size_t n = (1u<<30)/L; if (n>200000) n=200000;
  unsigned char *buf = malloc(n*L); for (size_t i=0;i<n*L;i++) buf[i]=(unsigned char)(i*2654435761u>>24);
  unsigned char d[16]; unsigned acc=0;
  for (int rep=0; rep<3; rep++){
    double t0=now();
    for (size_t i=0;i<n;i++){ struct MD5Context c; MD5Init(&c); MD5Update(&c, buf+i*L, L); MD5Final(d,&c); acc+=d[0]; }
    double t=now()-t0; printf("len %zu: %.3f GiB/s (%.1f ns/msg)\n", L, n*L/t/(1<<30), t/n*1e9);
  }
  return acc==12345;
}
