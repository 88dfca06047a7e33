/* CPU model (round 6): how often an ITB match reuses the previous match offset
 * (the last one or the last two), and in how many one-wave-encoder windows every
 * path match does -- i.e. how often a candidate predicted from the last offset
 * could be loaded with the dictionary probe.  Greedy parse restated from
 * oracle/lzo1x_oracle.c (lib/minilzo.c:2922-3157), windows as in
 * scripts/dbg/enc_empty_sim.c.  gcc -O2 -o /tmp/p scripts/dbg/enc_pred_sim.c &&
 * /tmp/p FILE (raw concatenated 64 KiB blocks). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
enum { SLOTS = 1u << 14, FAR = 0xBFFF, NEAR = 0x0800, GUARD = 13, WAVE = 64, PATHMAX = 6 };
static uint32_t h1_of(const uint8_t *p){uint32_t v=((((uint32_t)p[3]<<6)^p[2])<<5)^p[1];v=(v<<5)^p[0];return((v*33u)>>5)&(SLOTS-1);}
static uint32_t h2_of(uint32_t h){return (h&0x7FFu)^0x201Fu;}
static double win, allpred, allpred2, matches, pred1, pred2;
static void block(const uint8_t *in, size_t n){
  static uint32_t dict[SLOTS]; memset(dict,0,sizeof dict);
  size_t ip_end=n-GUARD, ip=4, dlast=0, dlast2=0;
  while(ip<ip_end){
    win++; size_t wend=ip+WAVE; int nm=0, ok_all=1, ok_all2=1;
    while(ip<ip_end&&ip<wend&&nm<PATHMAX){
      uint32_t slot=h1_of(in+ip),cand=dict[slot]; size_t c=0,off=0; int ok=0;
      if(cand&&ip-(cand-1)<=FAR){c=cand-1;off=ip-c;if(off<=NEAR||in[c+3]==in[ip+3])ok=1;else{slot=h2_of(slot);cand=dict[slot];if(cand&&ip-(cand-1)<=FAR){c=cand-1;off=ip-c;if(off<=NEAR||in[c+3]==in[ip+3])ok=1;}}}
      if(ok&&!(in[c]==in[ip]&&in[c+1]==in[ip+1]&&in[c+2]==in[ip+2]))ok=0;
      dict[slot]=ip+1;
      if(!ok){ip++;continue;}
      matches++;
      int p1 = off==dlast, p2 = off==dlast || off==dlast2;
      pred1+=p1; pred2+=p2; if(!p1) ok_all=0; if(!p2) ok_all2=0;
      if(off!=dlast){dlast2=dlast; dlast=off;}
      size_t len=3; while(ip+len<n&&in[c+len]==in[ip+len])len++; ip+=len; nm++;
    }
    allpred+=ok_all; allpred2+=ok_all2;
  }
}
int main(int argc,char**argv){ FILE*f=fopen(argv[1],"rb"); size_t bs=65536; uint8_t*buf=malloc(bs); size_t nb=0;
  while(fread(buf,1,bs,f)==bs){block(buf,bs);nb++;}
  printf("matches/block %.0f: offset == last %.1f%%, in last two %.1f%%; windows whose path matches are all predicted: %.1f%% / %.1f%%\n",
    matches/nb,100*pred1/matches,100*pred2/matches,100*allpred/win,100*allpred2/win);}
