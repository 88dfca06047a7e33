/* CPU model (round 6): claim conflicts of the one-wave encoder -- path lanes of a
 * window reading a slot an earlier path lane of the same window wrote (what the
 * kernel resolves by forwarding rounds) -- per window, their writer distance,
 * and how often that writer is simply the nearest lower lane with the same
 * primary hash (a conflict predictable before the walk).  Windows as in
 * scripts/dbg/enc_empty_sim.c.  gcc -O2 -o /tmp/c scripts/dbg/enc_conflict_sim.c &&
 * /tmp/c FILE (raw concatenated 64 KiB blocks) */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
enum { SLOTS = 1u << 14, FAR = 0xBFFF, NEAR = 0x0800, GUARD = 13, WAVE = 64, PATHMAX = 6 };
static uint32_t h1_of(const uint8_t *p){uint32_t v=((((uint32_t)p[3]<<6)^p[2])<<5)^p[1];v=(v<<5)^p[0];return((v*33u)>>5)&(SLOTS-1);}
static uint32_t h2_of(uint32_t h){return (h&0x7FFu)^0x201Fu;}
static double bok, win, conf, confwin, conf_match, conf_dist[5], pathlanes;
static void block(const uint8_t *in, size_t n){
  static uint32_t dict[SLOTS]; memset(dict,0,sizeof dict);
  size_t ip_end=n-GUARD, ip=4;
  while(ip<ip_end){
    win++; size_t ws=ip, wend=ip+WAVE; int nm=0; int wconf=0;
    static int32_t wslot_pos[SLOTS]; // position in this window that wrote the slot, -1 none
    static int touched[256]; int nt=0;
    while(ip<ip_end&&ip<wend&&nm<PATHMAX){
      uint32_t a=h1_of(in+ip), b=h2_of(a);
      // conflict: h1 (or h2 if used) written earlier in this window
      uint32_t slot=a,cand=dict[slot]; size_t c=0,off=0; int ok=0, used2=0;
      if(cand&&ip-(cand-1)<=FAR){c=cand-1;off=ip-c;if(off<=NEAR||in[c+3]==in[ip+3])ok=1;else{used2=1;slot=b;cand=dict[slot];if(cand&&ip-(cand-1)<=FAR){c=cand-1;off=ip-c;if(off<=NEAR||in[c+3]==in[ip+3])ok=1;}}}
      int isconf = (wslot_pos[a]>0) || (used2 && wslot_pos[b]>0);
      if(ok&&!(in[c]==in[ip]&&in[c+1]==in[ip+1]&&in[c+2]==in[ip+2]))ok=0;
      pathlanes++;
      if(isconf){
        /* nearest lower lane of the window with the same h1 */
        int q=-1; for(size_t y=ip; y-- > ws;){ if(h1_of(in+y)==a){q=(int)y;break;} }
        int via1 = wslot_pos[a]>0;
        if(via1 && q>=0 && (size_t)(wslot_pos[a]-1)==(size_t)q && !(a>=0x2000&&a<0x2800)) bok++;
        conf++; wconf++; if(ok) conf_match++; size_t d = ip - (size_t)(wslot_pos[a]>0? wslot_pos[a]-1 : wslot_pos[b]-1); int k = d<=1?0:d<=4?1:d<=16?2:d<=32?3:4; conf_dist[k]++;}
      dict[slot]=ip+1; if(!wslot_pos[slot] && nt<256) touched[nt++]=slot; wslot_pos[slot]=ip+1;
      if(!ok){ip++;continue;}
      size_t len=3; while(ip+len<n&&in[c+len]==in[ip+len])len++; ip+=len; nm++;
    }
    for(int i=0;i<nt;i++) wslot_pos[touched[i]]=0;
    confwin += wconf>0;
  }
}
int main(int argc,char**argv){ FILE*f=fopen(argv[1],"rb"); size_t bs=65536; uint8_t*buf=malloc(bs); size_t nb=0;
  while(fread(buf,1,bs,f)==bs){block(buf,bs);nb++;}
  printf("windows/block %.0f, path lanes/window %.1f, conflicts/block %.0f (%.2f per window), windows with any %.1f%%, conflicting lanes that match %.1f%%\n", win/nb, pathlanes/win, conf/nb, conf/win, 100*confwin/win, 100*conf_match/conf);
  printf("conflicts whose writer is the nearest lower same-h1 lane (h1 outside the secondary range): %.1f%%\n",100*bok/conf); printf("distance to the writer: 1 %.0f%%, 2-4 %.0f%%, 5-16 %.0f%%, 17-32 %.0f%%, 33+ %.0f%%\n", 100*conf_dist[0]/conf,100*conf_dist[1]/conf,100*conf_dist[2]/conf,100*conf_dist[3]/conf,100*conf_dist[4]/conf);}
