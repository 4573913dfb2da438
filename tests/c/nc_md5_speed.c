/* Host nc_MD5 speed (netcache cache-key digests, diskcache.c:3443-3452):
 * nc_MD5Init/Update/Final per key, linked against libmd5hip's nc_md5.c or
 * against the reference netcache/netcache/md5.c compiled in place, by
 * scripts/nc_md5_speed.sh.  Bench tool, not a test. */
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <time.h>
typedef struct { unsigned long i[2]; unsigned long buf[4]; unsigned char in[64]; unsigned char digest[16]; } nc_MD5_CTX;
void nc_MD5Init(nc_MD5_CTX *); void nc_MD5Update(nc_MD5_CTX *, unsigned char *, unsigned int); void nc_MD5Final(nc_MD5_CTX *);
static double now(void){struct timespec t; clock_gettime(CLOCK_MONOTONIC,&t); return t.tv_sec+t.tv_nsec*1e-9;}
int main(int argc, char **argv){
  size_t L = argc>1? strtoul(argv[1],0,0):128; size_t n = 1000000;
  unsigned char *buf = malloc(n*L); for (size_t i=0;i<n*L;i++) buf[i]=(unsigned char)(i*2654435761u>>24);
  unsigned acc=0; double best=1e30;
  for (int rep=0; rep<5; rep++){
    double t0=now();
    for (size_t i=0;i<n;i++){ nc_MD5_CTX c; nc_MD5Init(&c); nc_MD5Update(&c, buf+i*L, (unsigned)L); nc_MD5Final(&c); acc+=c.digest[0]; }
    double t=now()-t0; if (t<best) best=t;
  }
  printf("len %zu: %.1f ns/key, %.3f GiB/s (best of 5, %zu keys, check %u)\n", L, best/n*1e9, n*L/best/(1<<30), n, acc);
  return 0;
}
