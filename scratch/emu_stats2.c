#include <stdint.h>
#include <stdlib.h>
#include <string.h>
static uint32_t head_be(const uint8_t*b,uint32_t p,uint32_t len){uint32_t v=0;for(int k=0;k<4;k++) if(p+k<len) v|=(uint32_t)b[p+k]<<(8*k); return __builtin_bswap32(v);}
static uint32_t w4(const uint8_t*W,uint32_t x){uint32_t v; memcpy(&v,W+x,4); return v;}
/* out: hops, pass, improve, pass_first4, pass_tail4, hops_first4, mbytes, iters4 (matchlen loop iterations at 4B), iters8 */
void stats2(const uint8_t* blk, uint32_t len, uint32_t chain, uint32_t nice, double* out)
{
    uint16_t* p4=calloc(len+1,2); int32_t* h4=malloc(65536*4); for(int i=0;i<65536;i++)h4[i]=-1;
    for(uint32_t p=0;p<len;p++){ uint32_t hd=p?head_be(blk,p,len):0; uint32_t a=p?(hd*0x1e35a7bdu)>>16:0; p4[p]=h4[a]<0?0:p-h4[a]; h4[a]=p; }
    uint8_t* W=calloc(len+600,1); memcpy(W,blk,len);
    double o[12]={0};
    for(uint32_t p=0;p<len;p++){ uint32_t cl=2,it=0,d=p4[p],q=p-d;
        for(;;){ if(it>=chain||d==0||p-q>=32768) break; o[0]++;
            int f4 = w4(W,p)==w4(W,q); o[5]+=f4;
            if(W[q+cl]==W[p+cl]){ o[1]++; o[3]+=f4; o[4]+= (cl>=3 && q>=3) ? (w4(W,p+cl-3)==w4(W,q+cl-3)) : 1;
                uint32_t m=0; while(m<258&&W[p+m]==W[q+m])m++; o[6]+=m; o[7]+= m/4+1; o[8]+=m/8+1;
                if(m>cl){o[2]++; cl=m; if(cl>=nice)break;}}
            it++; d=p4[q]; q-=d; } }
    for(int i=0;i<9;i++) out[i]=o[i]/len;
    free(p4);free(h4);free(W);
}
