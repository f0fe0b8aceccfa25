#include <stdint.h>
#include <stdlib.h>
#include <string.h>
static uint32_t head_be(const uint8_t*b,uint32_t p,uint32_t len){uint32_t v=0;for(int k=0;k<4;k++) if(p+k<len) v|=(uint32_t)b[p+k]<<(8*k); return __builtin_bswap32(v);}
/* out: hops4 (baseline), hops_skip (4-chain until cl>=K-1, then K-gram chain), fullwalk fraction */
void skipstats(const uint8_t* blk, uint32_t len, uint32_t chain, uint32_t nice, uint32_t K, double* out)
{
    uint16_t* p4=calloc(len+1,2); int32_t* h4=malloc(65536*4); for(int i=0;i<65536;i++)h4[i]=-1;
    uint32_t* rank=calloc(len+1,4); uint32_t* cntb=calloc(65536,4);
    for(uint32_t p=0;p<len;p++){ uint32_t hd=p?head_be(blk,p,len):0; uint32_t a=p?(hd*0x1e35a7bdu)>>16:0; p4[p]=h4[a]<0?0:p-h4[a]; h4[a]=p; rank[p]=cntb[a]++; }
    uint8_t* W=calloc(len+600,1); memcpy(W,blk,len);
    /* K-gram chain: previous position with identical K bytes (exact, via simple hash map of K-gram -> last pos) */
    int32_t* pk=malloc((len+1)*4);
    { uint32_t HS=1u<<20; int32_t* hk=malloc(HS*4); for(uint32_t i=0;i<HS;i++)hk[i]=-1;
      for(uint32_t p=0;p<len;p++){ uint64_t h=1469598103934665603ull; for(uint32_t k=0;k<K;k++){h^=W[p+k]; h*=1099511628211ull;} uint32_t s=(uint32_t)(h>>44);
        /* resolve collisions by probing */
        int32_t q=hk[s]; pk[p]=-1;
        while(q>=0 && memcmp(W+q,W+p,K)!=0){ s=(s+1)&(HS-1); q=hk[s]; }
        pk[p]=q; hk[s]=p; }
      free(hk); }
    double hb=0, hs=0;
    for(uint32_t p=0;p<len;p++){
        /* baseline */
        uint32_t cl=2,it=0,d=p4[p],q=p-d;
        for(;;){ if(it>=chain||d==0||p-q>=32768) break; hb++;
            if(W[q+cl]==W[p+cl]){ uint32_t m=0; while(m<258&&W[p+m]==W[q+m])m++; if(m>cl){cl=m; if(cl>=nice)break;}}
            it++; d=p4[q]; q-=d; }
        /* skip version */
        cl=2; it=0; d=p4[p]; q=p-d; int onk=0;
        for(;;){
            if(!onk){ if(it>=chain||d==0||p-q>=32768) break; }
            else { if(rank[p]-rank[q] > chain || p-q>=32768) break; }
            hs++;
            if(W[q+cl]==W[p+cl]){ uint32_t m=0; while(m<258&&W[p+m]==W[q+m])m++; if(m>cl){cl=m; if(cl>=nice)break;}}
            if(!onk && cl>=K-1){ onk=1; }
            if(!onk){ it++; d=p4[q]; q-=d; }
            else { int32_t qq; /* next candidate sharing K bytes with p, below q: walk K-chain from q */
                   qq = (memcmp(W+q,W+p,K)==0) ? pk[q] : -1;
                   if(qq<0){ /* q itself doesn't share K bytes: find the K-chain entry below q starting from p */
                       qq=pk[p]; while(qq>=0 && (uint32_t)qq>=q) qq=pk[qq]; }
                   if(qq<0) break; q=(uint32_t)qq; }
        }
    }
    out[0]=hb/len; out[1]=hs/len;
    free(p4);free(h4);free(W);free(pk);free(rank);free(cntb);
}
