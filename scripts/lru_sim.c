// LRU model of the per-XCD L2 for the light kernel: workgroups of 8 rows dealt
// round-robin to 8 XCDs, each XCD an LRU of `cap` X row-slices (4 MB / 512 B
// = 8192 at 128-float slices).  Used by scripts/locality_sim.py.
// usage: lru_sim n nnz order.bin row_ptr.bin col.bin cap xcds rows_per_wg [n_order]
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
// usage: lru n nnz rows_file rp_file ci_file cap xcds rows_per_wg
int main(int argc,char**argv){
  long n=atol(argv[1]), nnz=atol(argv[2]);
  int cap=atoi(argv[6]), X=atoi(argv[7]), rpw=atoi(argv[8]);
  long no=argc>9?atol(argv[9]):n;  /* rows processed: the first no entries of order */
  int32_t*order=malloc(no*4),*rp=malloc((n+1)*4),*ci=malloc(nnz*4);
  FILE*f=fopen(argv[3],"rb");fread(order,4,no,f);fclose(f);
  f=fopen(argv[4],"rb");fread(rp,4,n+1,f);fclose(f);
  f=fopen(argv[5],"rb");fread(ci,4,nnz,f);fclose(f);
  // per-XCD LRU: prev/next arrays over columns
  int32_t *prv=malloc((size_t)X*n*4),*nxt=malloc((size_t)X*n*4); char*in=calloc((size_t)X*n,1);
  int32_t head[64],tail[64],size[64]; for(int x=0;x<X;x++){head[x]=tail[x]=-1;size[x]=0;}
  long hits=0,acc=0;
  long nwg=(no+rpw-1)/rpw;
  for(long w=0;w<nwg;w++){ int x=w%X; int32_t*P=prv+(size_t)x*n,*N=nxt+(size_t)x*n; char*I=in+(size_t)x*n;
    for(long r=w*rpw;r<(w+1)*rpw && r<no;r++){ int32_t row=order[r];
      for(int k=rp[row];k<rp[row+1];k++){ int c=ci[k]; acc++;
        if(I[c]){ hits++; // move to front
          if(head[x]!=c){ int p=P[c],q=N[c]; N[p]=q; if(q>=0)P[q]=p; else tail[x]=p; P[c]=-1;N[c]=head[x];P[head[x]]=c;head[x]=c;}
        } else { I[c]=1; P[c]=-1; N[c]=head[x]; if(head[x]>=0)P[head[x]]=c; head[x]=c; if(tail[x]<0)tail[x]=c; size[x]++;
          if(size[x]>cap){ int t=tail[x]; int p=P[t]; I[t]=0; tail[x]=p; N[p]=-1; size[x]--; } }
      }}}
  printf("hit_rate %.4f accesses %ld\n",(double)hits/acc,acc);
  return 0;}
