/* CPU model (round 6): a direct-mapped LDS cache of C recent dictionary puts
 * (index (slot ^ slot >> 9) mod C): share of probe loads it serves, windows whose
 * probes it serves entirely, dictionary lines per window left, and puts that
 * evict another slot (the global stores left).  Windows as in
 * scripts/dbg/enc_empty_sim.c.  gcc -O2 -o /tmp/w scripts/dbg/enc_wbc_sim.c &&
 * /tmp/w FILE 65536 C */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
enum { SLOTS = 1u << 14, FAR = 0xBFFF, NEAR = 0x0800, GUARD = 13, WAVE = 64, PATHMAX = 6 };
static uint32_t h1_of(const uint8_t *p){uint32_t v=((((uint32_t)p[3]<<6)^p[2])<<5)^p[1];v=(v<<5)^p[0];return((v*33u)>>5)&(SLOTS-1);}
static uint32_t h2_of(uint32_t h){return (h&0x7FFu)^0x201Fu;}
static int C;
static double win, need, served, allserved, lines_need, lines_left, nput, evict;
static uint32_t cidx(uint32_t s){ return (s ^ (s >> 9)) & (C - 1); }
static void block(const uint8_t *in, size_t n){
  static uint32_t dict[SLOTS]; static uint8_t wr[SLOTS]; static int32_t ck[1<<16];
  memset(dict,0,sizeof dict); memset(wr,0,sizeof wr); for(int i=0;i<C;i++) ck[i]=-1;
  size_t ip_end=n-GUARD, ip=4;
  while(ip<ip_end){
    win++; int any=0; uint8_t ln[256]={0}, ll[256]={0};
    for(size_t p=ip;p<ip+WAVE&&(p<ip_end||p==ip);p++){
      uint32_t a=h1_of(in+p), b=h2_of(a);
      if(wr[a]){ need++; ln[a/64]=1; if(ck[cidx(a)]==(int32_t)a) served++; else {any=1; ll[a/64]=1;} }
      if(wr[a]&&wr[b]){ need++; ln[b/64]=1; if(ck[cidx(b)]==(int32_t)b) served++; else {any=1; ll[b/64]=1;} }
    }
    allserved+=!any; for(int i=0;i<256;i++){lines_need+=ln[i]; lines_left+=ll[i];}
    size_t wend=ip+WAVE; int nm=0;
    while(ip<ip_end&&ip<wend&&nm<PATHMAX){
      uint32_t slot=h1_of(in+ip),cand=dict[slot]; size_t c=0,off; int ok=0;
      if(cand&&ip-(cand-1)<=FAR){c=cand-1;off=ip-c;if(off<=NEAR||in[c+3]==in[ip+3])ok=1;else{slot=h2_of(slot);cand=dict[slot];if(cand&&ip-(cand-1)<=FAR){c=cand-1;off=ip-c;if(off<=NEAR||in[c+3]==in[ip+3])ok=1;}}}
      if(ok&&!(in[c]==in[ip]&&in[c+1]==in[ip+1]&&in[c+2]==in[ip+2]))ok=0;
      dict[slot]=ip+1; wr[slot]=1; nput++; if(ck[cidx(slot)]>=0 && ck[cidx(slot)]!=(int32_t)slot) evict++; ck[cidx(slot)]=slot;
      if(!ok){ip++;continue;}
      size_t len=3; while(ip+len<n&&in[c+len]==in[ip+len])len++; ip+=len; nm++;
    }
  }
}
int main(int argc,char**argv){ C=atoi(argv[3]); FILE*f=fopen(argv[1],"rb"); size_t bs=strtoul(argv[2],0,0); uint8_t*buf=malloc(bs); size_t nb=0;
  while(fread(buf,1,bs,f)==bs){block(buf,bs);nb++;}
  printf("nput/block %.0f, global stores (evictions) %.1f%%; ",nput/nb,100*evict/nput); printf("C=%d: probe loads served %.1f%%, windows all served %.1f%%, dict lines/window %.1f -> %.1f\n",C,100*served/need,100*allserved/win,lines_need/win,lines_left/win);}
