/*
 * decomp_emu.c -- CPU model of the GPU decomposition of the level 6-9
 * deflater (TEST SUPPORT ONLY): k_chains (per-position chain links),
 * k_match (one chain walk per position with a running threshold of 2,
 * recording the full- and half-budget results and the 3-byte candidate) and
 * k_parse (lazy parse over the records, including the held step whose
 * threshold reaches `nice`).  tests/test_decomposition.py checks that this
 * decomposition reproduces the oracle's token stream, i.e. that the
 * restructuring argued in DESIGN.md is exact, without a GPU.
 *
 * emu_slice = 1 models the block-mode chain representation of round 6: no
 * links, but the block's positions sorted by (hash-4 bucket, position) -- S --
 * with each position's rank r(p) in S and count c(p) of earlier positions in
 * its bucket.  Position p's chain is then the contiguous slice S[r-1],
 * S[r-2], ..., S[r-c] (newest first), cut at 32 KiB as before; k_chains<4>
 * builds S by a counting sort and k_match reads the slice without a pointer
 * chase.  Both walks must give the same records.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static uint32_t lsym(uint32_t len){uint32_t x=len-3; if(len==258)return 28; if(x<8)return x; uint32_t e=29-__builtin_clz(x); return 4*e+4+((x>>e)&3);}
static int ilog2(uint32_t x){return 31-__builtin_clz(x);}
static uint32_t head_be(const uint8_t*b,uint32_t p,uint32_t len){uint32_t v=0;for(int k=0;k<4;k++) if(p+k<len) v|=(uint32_t)b[p+k]<<(8*k); return __builtin_bswap32(v);}
unsigned long slowcalls=0;
int emu_slice=0;
/* the j-th candidate (1-based) of p, or -1 past its chain; candidates are
 * asked for in order j = 1, 2, ... (the link walk steps from *q) */
static int64_t cand(const uint16_t*p4,const uint16_t*S,const uint32_t*R,const uint32_t*C,uint32_t p,uint32_t j,uint32_t*q){
    if(emu_slice){ if(j>C[p]) return -1; *q=S[R[p]-j]; return 0; }
    uint32_t x=j==1?p:*q; uint32_t d=p4[x]; if(!d) return -1; *q=x-d; return 0; }  /* *q: candidate j-1 */
int emu(const uint8_t* blk, uint32_t len, int level, uint32_t* tok, uint32_t* ntok_out, uint32_t* dbends, uint32_t* ndb_out)
{
    uint32_t good,nice,chain,lzcap;
    switch(level){case 6: good=16;nice=16;chain=48;lzcap=65536;break; case 7: good=32;nice=64;chain=128;lzcap=65536;break;
      case 8: good=64;nice=128;chain=320;lzcap=131072;break; default: good=192;nice=256;chain=512;lzcap=131072;}
    uint16_t* p4=calloc(len+1,2); uint16_t* p3=calloc(len+1,2); uint64_t* rec=calloc(len+1,8); uint32_t half=chain>>1;
    int32_t* h4=malloc(65536*4); int32_t* h3=malloc(16384*4);
    for(int i=0;i<65536;i++)h4[i]=-1; for(int i=0;i<16384;i++)h3[i]=-1;
    uint32_t* A=calloc(len+1,4); uint32_t* R=calloc(len+1,4); uint32_t* C=calloc(len+1,4); uint16_t* S=calloc(len+1,2);
    uint32_t* cnt=calloc(65536,4);
    for(uint32_t p=0;p<len;p++){ uint32_t hd=p?head_be(blk,p,len):0; uint32_t a=p?(hd*0x1e35a7bdu)>>16:0, b=p?((hd>>8)*0x1e35a7bdu)>>18:0;
        p4[p]= h4[a]<0?0:p-h4[a]; h4[a]=p; p3[p]= h3[b]<0?0:h3[b]; h3[b]=p; A[p]=a; C[p]=cnt[a]++; }
    /* counting sort by bucket: exclusive scan of the counts, then scatter */
    for(uint32_t h=0,run=0;h<65536;h++){ uint32_t t=cnt[h]; cnt[h]=run; run+=t; }
    for(uint32_t p=0;p<len;p++){ R[p]=cnt[A[p]]+C[p]; S[R[p]]=(uint16_t)p; }
    uint8_t* W=calloc(len+600,1); memcpy(W,blk,len);
    for(uint32_t p=0;p<len;p++){
        uint32_t cl=2,co=0,l24=0,o24=0,it=0; int have24=0; uint32_t q=0, j=1;
        for(;;){ if(it>=chain||cand(p4,S,R,C,p,j,&q)<0||p-q>=32768)break; int fin=0;
            if(W[q+cl]==W[p+cl]){uint32_t m=0; while(m<258&&W[p+m]==W[q+m])m++; if(m>cl){cl=m;co=p-q;if(cl>=nice)fin=1;}}
            if(fin)break; it++; if(it==half){l24=cl;o24=co;have24=1;} j++; }
        if(!have24){l24=cl;o24=co;}
        uint32_t rem=len-p; uint32_t t48=cl>=3?(cl<rem?cl:rem):0, t24=l24>=3?(l24<rem?l24:rem):0, s3=0;
        if(cl<3){ uint32_t n3=p3[p]; if(n3){ uint32_t noff=(p-n3)&0xffff; if(noff<=32768&&noff){ if(W[p]==W[p-noff]&&W[p+1]==W[p-noff+1]&&W[p+2]==W[p-noff+2]) s3=noff; else { uint32_t r=n3+((p-n3)&~16383u); uint32_t n3b=p3[r]; if(n3b){noff=(p-n3b)&0xffff; if(noff<=32768&&noff&&W[p]==W[p-noff]&&W[p+1]==W[p-noff+1]&&W[p+2]==W[p-noff+2]) s3=noff;}}}} if(s3>8192)s3=0;}
        rec[p]=(uint64_t)t48|((uint64_t)(t48?co:0)<<9)|((uint64_t)t24<<24)|((uint64_t)(t24?o24:0)<<33)|((uint64_t)s3<<48);
    }
    uint32_t curr[32]={0},prv[32]={0},obscount=0,newcount=0,obstotal=0,cur=0,nt=0,slots=0,ndb=0,hm=0,hl=0,ho=0,ds=0,lastc=0;
    while(cur<len){ uint64_t r=rec[cur]; uint32_t c=blk[cur]; uint32_t l48=r&511,o48=(r>>9)&0x7fff;
        if(!hm){ uint32_t ml=l48,mo=o48,s3=r>>48; if(l48==0&&ds&&s3&&cur+3<=len){ml=3;mo=s3;} if(ml==3&&mo>8192)ml=2;
            if(ml>=3){ if(ml>=good){tok[nt++]=0x80000000u|(ml<<16)|mo;slots+=3;curr[16+(lsym(ml)>>1)]++;newcount++;obstotal+=ml;cur+=ml-1;} else {hm=1;hl=ml;ho=mo;} }
            else { tok[nt++]=c;slots++;curr[c>>4]++;newcount++;obstotal++; } }
        else { uint32_t l24=(r>>24)&511,o24=(r>>33)&0x7fff; uint32_t ml=hl>=4?l24:l48, mo=hl>=4?o24:o48; int acc=0;
            if(hl-1>=nice){ /* first candidate (half budget) longer than L0 */
                uint32_t L0=hl-1, q=0, it=0; ml=0; mo=0; slowcalls++;
                while(it<half && cand(p4,S,R,C,cur,it+1,&q)==0 && cur-q<32768){ if(W[q+L0]==W[cur+L0]){uint32_t mm=0; while(mm<258&&W[cur+mm]==W[q+mm])mm++; if(mm>L0){ml=mm<len-cur?mm:len-cur;mo=cur-q;break;}} it++; }
            }
            if(ml>=hl){int dl=ml-hl; acc=dl>4||(dl*4+ilog2(ho)-ilog2(mo))>=2;}
            if(acc){tok[nt++]=lastc;slots++;curr[lastc>>4]++;newcount++;obstotal++;hl=ml;ho=mo;}
            else {tok[nt++]=0x80000000u|(hl<<16)|ho;slots+=3;curr[16+(lsym(hl)>>1)]++;newcount++;obstotal+=hl;cur+=hl-2;hm=0;} }
        lastc=c; cur++;
        if(slots+4>lzcap){dbends[ndb++]=nt;slots=0;memset(curr,0,128);memset(prv,0,128);obscount=newcount=obstotal=0;}
        else if(newcount>=512&&obstotal>=4096){ ds=curr[0]>=16; int split=0; if(obscount>0){uint32_t delta=0;for(int j=0;j<32;j++)delta+=prv[j]>curr[j]?prv[j]-curr[j]:curr[j]-prv[j]; split=delta>=320&&obstotal>=7168;}
            if(split){memset(curr,0,128);memset(prv,0,128);obscount=newcount=obstotal=0;dbends[ndb++]=nt;slots=0;}
            else{for(int j=0;j<32;j++){prv[j]=(prv[j]>>1)+(curr[j]>>1);curr[j]=0;}obscount+=newcount;newcount=0;} }
    }
    if(slots)dbends[ndb++]=nt;
    *ntok_out=nt;*ndb_out=ndb; free(p4);free(p3);free(rec);free(h4);free(h3);free(W); free(A);free(R);free(C);free(S);free(cnt); return 0;
}
